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
    """Linear scan of the kernel text, twice (the second pass models a loop back
    edge carrying loads issued at the end of a loop body into its head).  Pending
    asm loads complete in issue order: `s_waitcnt vmcnt(N)` retires all but the
    N most recent.  Labels do NOT reset the state (a ring's loads cross blocks)."""
    problems = []
    if re.search(r"s_set_gpr_idx_on|v_movrel|scratch_|buffer_store_dword .*off, s\[0:3\]", body):
        problems.append("dynamic GPR indexing or scratch access")
    lines = [l.strip() for l in body.split("\n")]
    pending = []  # [(regs, instr)] in issue order
    seen = set()
    for pas in range(2):
        for t in lines:
            if not t or t.startswith((";", ".")) or re.match(r"^\S+:$", t):
                continue
            m = re.match(r"(?:global|buffer)_load_dword(?:x\d)? (v\d+|v\[\d+:\d+\]),", t)
            if m:
                regs = _regs(m.group(1))
                pending = [(r, i) for r, i in pending if not (r & regs)]
                pending.append((regs, t))
                continue
            w = re.match(r"s_waitcnt .*vmcnt\((\d+)\)", t)
            if w:
                n = int(w.group(1))
                pending = pending[len(pending) - n:] if n < len(pending) else pending
                if n == 0:
                    pending = []
                continue
            parts = t.split(None, 1)
            if len(parts) < 2:
                continue
            ops = parts[1].split(",")
            store = parts[0].startswith(("global_store", "ds_write", "buffer_store", "flat_store"))
            srcs = _regs(parts[1]) if store else _regs(",".join(ops[1:]))
            dst = set() if store else _regs(ops[0])
            mad = re.match(r"v_mad_[ui]64_[ui]32 v\[(\d+):(\d+)\], [^,]+, [^,]+, [^,]+, v\[(\d+):(\d+)\]", t)
            if mad:  # the addend's high dword only reaches the result's high dword: taint it, do not flag
                hi_src, hi_dst = int(mad.group(4)), int(mad.group(2))
                hit = [ld for r, ld in pending if hi_src in r]
                if hit:
                    srcs = srcs - {hi_src}
                    dst = dst - {hi_dst}
                    pending = [(r - {hi_dst}, i) for r, i in pending if r - {hi_dst}] + [({hi_dst}, hit[0])]
            for regs, ld in pending:
                if regs & srcs and t not in seen:
                    seen.add(t)
                    problems.append(f"v{sorted(regs & srcs)} read before its wait: {t}  (load: {ld})")
            # a register overwritten by another instruction no longer holds the load's data
            pending = [(r - dst, i) for r, i in pending if r - dst]
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
