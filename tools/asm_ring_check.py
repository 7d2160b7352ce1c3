#!/usr/bin/env python3
"""Static check of the engine's hand-pipelined loads in compiled gfx950 assembly.

The kernels issue global loads as inline asm and wait for them with hand-counted
s_waitcnt vmcnt(N); the compiler does not know those loads are asynchronous, so
a register it copies (v_mov, s_set_gpr_idx, scratch spill) between the asm load
and its wait holds stale data.  check() reports, per basic block, instructions
that READ the destination of an asm global_load before a vmcnt wait, plus any
dynamic GPR indexing or scratch use in the kernel."""
import re
import sys


def _regs(s):
    out = set()
    for m in re.finditer(r"v\[(\d+):(\d+)\]|\bv(\d+)\b", s):
        if m.group(3):
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def kernels(text):
    """{symbol: body} of every kernel in an assembly file."""
    out = {}
    for m in re.finditer(r"^(_Z\w+):.*?$(.*?)s_endpgm", text, re.S | re.M):
        out[m.group(1)] = m.group(2)
    return out


def check(body):
    problems = []
    if re.search(r"s_set_gpr_idx_on|v_movrel|scratch_|buffer_store_dword .*off, s\[0:3\]", body):
        problems.append("dynamic GPR indexing or scratch access")
    pending = {}
    for l in body.split("\n"):
        t = l.strip()
        if not t or t.startswith(";"):
            continue
        if re.match(r"\.LBB|^\S+:", t):
            pending = {}
            continue
        m = re.match(r"global_load_dword (v\d+),", t)
        if m:
            pending[int(m.group(1)[1:])] = t
            continue
        if t.startswith("s_waitcnt") and "vmcnt" in t:
            pending = {}
            continue
        parts = t.split(None, 1)
        if len(parts) < 2:
            continue
        ops = parts[1].split(",")
        store = parts[0].startswith(("global_store", "ds_write", "buffer_store", "flat_store"))
        srcs = _regs(parts[1]) if store else _regs(",".join(ops[1:]))
        dst = set() if store else _regs(ops[0])
        for v in list(pending):
            if v in srcs:
                problems.append(f"v{v} read before its wait: {t}")
            elif v in dst:
                del pending[v]
    return problems


if __name__ == "__main__":
    text = open(sys.argv[1]).read()
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    bad = 0
    for sym, body in kernels(text).items():
        if sub in sym:
            p = check(body)
            bad += len(p)
            for x in p[:5]:
                print(sym, x)
    print("problems", bad)
    sys.exit(1 if bad else 0)
