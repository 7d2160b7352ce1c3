#!/usr/bin/env python3
"""Static check of the engine's hand-pipelined loads in compiled gfx950 assembly.

The kernels issue their HBM loads as inline asm and wait for them with
hand-counted `s_waitcnt vmcnt(N)`; the compiler does not know those loads are
asynchronous, so a register it copies (v_mov, a select, a spill) between an asm
load and the wait that covers it holds stale data, and a register it writes
while a load into it is in flight is clobbered when the load lands.

check() runs a forward dataflow analysis over the kernel's control-flow graph
(basic blocks from labels / `; %bb.N:` markers, edges from s_branch /
s_cbranch_* and fall-through).  The state maps every VGPR with a load in
flight to the minimum, over all paths, of the number of loads issued after it.
Loads complete in issue order, so `s_waitcnt vmcnt(N)` retires every load with
at least N younger loads.  Stores are not counted as younger operations
(conservative).  Reported: any read of an in-flight register, any write to
one by a non-load instruction, dynamic GPR indexing and scratch access.
`s_cbranch_execz` edges are not followed (their fall-through executes the same
instructions with EXEC = 0).
"""
import re
import sys

_LOAD = re.compile(r"(?:global|buffer|flat)_load_(?:dword(?:x\d)?|ubyte|ushort|sbyte|sshort)\w*\s+([va]\d+|[va]\[\d+:\d+\])")
_WAIT = re.compile(r"s_waitcnt\b.*\bvmcnt\((\d+)\)")
_LABEL = re.compile(r"^(\.LBB\w+):")
_BB = re.compile(r"^;\s*%bb\.\d+:")
_BR = re.compile(r"^s_(c?branch)\w*\s+(\.LBB\w+)")


def _regs(s):
    """VGPR numbers in an operand string; AGPR n is reported as 1000 + n."""
    out = set()
    for m in re.finditer(r"\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b", s):
        if m.group(5):
            out.add(int(m.group(5)) + (1000 if m.group(4) == "a" else 0))
        else:
            base = 1000 if m.group(1) == "a" else 0
            out.update(range(base + int(m.group(2)), base + int(m.group(3)) + 1))
    return out


def kernels(text):
    """{symbol: body} of every kernel in an assembly file."""
    out = {}
    for m in re.finditer(r"^(_Z\w+):.*?$(.*?)s_endpgm", text, re.S | re.M):
        out[m.group(1)] = m.group(2) + "\ns_endpgm"
    return out


def _blocks(body):
    """[(name, [instr...], [successor names])] in text order."""
    blocks, cur, name, n = [], [], "entry", 0
    for raw in body.split("\n"):
        t = raw.strip()
        if not t:
            continue
        lab = _LABEL.match(t)
        if lab or _BB.match(t):
            blocks.append([name, cur])
            name = lab.group(1) if lab else f"_bb{n}"
            n += 1
            cur = []
            continue
        if t.startswith((";", ".")):
            continue
        cur.append(t.split(";")[0].strip())
    blocks.append([name, cur])
    out = []
    for i, (nm, ins) in enumerate(blocks):
        succ, falls = [], True
        for t in ins:
            b = _BR.match(t)
            if b:
                # s_cbranch_execz skips a region whose lanes are all inactive; the
                # fall-through runs the same instructions (and waits) with EXEC = 0,
                # so it covers the skip: following only it removes infeasible paths
                # around this engine's uniform loops (EXEC is never zero there)
                if t.startswith("s_cbranch_execz"):
                    continue
                succ.append(b.group(2))
                if b.group(1) == "branch":
                    falls = False
            if t.startswith(("s_endpgm", "s_setpc", "s_trap")):
                falls = False
        if falls and i + 1 < len(blocks):
            succ.append(blocks[i + 1][0])
        out.append((nm, ins, succ))
    return out


def _step(state, t, problems, where):
    """Transfer one instruction; state = {reg: (younger_loads, load_text)}."""
    m = _LOAD.match(t)
    if m:
        regs = _regs(m.group(1))
        for r in _regs(t[m.end():]) & set(state):
            problems.add(f"v{r} (in flight) used as a load operand: {t}  [{where}]")
        new = {r: (y + 1, ld) for r, (y, ld) in state.items() if r not in regs}
        for r in regs:
            new[r] = (0, t)
        return new
    w = _WAIT.match(t)
    if w:
        n = int(w.group(1))
        return {r: v for r, v in state.items() if v[0] < n}
    parts = t.split(None, 1)
    if len(parts) < 2 or not state:
        return state
    op, rest = parts
    ops = rest.split(",")
    store = op.startswith(("global_store", "buffer_store", "flat_store", "global_atomic", "ds_write", "ds_bpermute"))
    srcs = _regs(rest) if store else _regs(",".join(ops[1:]))
    dst = set() if store else _regs(ops[0])
    if op.startswith(("v_mad_u64_u32", "v_mad_i64_i32")):
        # the addend's high dword only reaches the result's high dword: taint it instead
        mad = re.match(r"v\[(\d+):(\d+)\],[^,]+,[^,]+,[^,]+,\s*v\[(\d+):(\d+)\]", rest)
        if mad and int(mad.group(4)) in state:
            hi_src, hi_dst = int(mad.group(4)), int(mad.group(2))
            srcs = srcs - {hi_src}
            taint = state[hi_src]
            state = {r: v for r, v in state.items() if r not in dst}
            state[hi_dst] = taint
            dst = set()
    for r in sorted(srcs & set(state)):
        problems.add(f"v{r} read before its wait: {t}  (load: {state[r][1]})  [{where}]")
    for r in sorted(dst & set(state)):
        problems.add(f"v{r} written while a load into it is in flight: {t}  (load: {state[r][1]})  [{where}]")
    if dst & set(state):
        state = {r: v for r, v in state.items() if r not in dst}
    return state


def check_local(body):
    """Block-local variant (state reset at every label): no cross-block paths, so
    no infeasible ones either.  Used for the branchy kernels (stream, gv4) whose
    CFG has many SGPR-correlated branches the dataflow analysis cannot prune;
    it still catches a ring register copied or clobbered inside a block."""
    problems = set()
    if re.search(r"s_set_gpr_idx_on|v_movrel|scratch_|buffer_store_dword .*off, s\[0:3\]", body):
        problems.add("dynamic GPR indexing or scratch access")
    for nm, ins, _ in _blocks(body):
        st = {}
        for t in ins:
            st = _step(st, t, problems, nm)
    return sorted(problems)


def check_pinned(body, first=224, last=255):
    """For kernels whose ring lives in PINNED registers v[first..last] above the
    compiler's budget (general_v4.hip): no compiler-generated instruction may
    touch them, i.e. every reference must sit inside an inline-asm region
    (;;#ASMSTART .. ;;#ASMEND), where the ring protocol is written by hand."""
    problems, in_asm = set(), False
    pinned = set(range(first, last + 1))
    for raw in body.split("\n"):
        t = raw.strip()
        if t.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if t.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if in_asm or not t or t.startswith((";", ".")):
            continue
        hit = _regs(t.split(";")[0]) & pinned
        if hit:
            problems.add(f"compiler code touches pinned ring register(s) {sorted(hit)[:4]}: {t}")
    if re.search(r"s_set_gpr_idx_on|v_movrel|scratch_", body):
        problems.add("dynamic GPR indexing or scratch access")
    return sorted(problems)


def _merge(a, b):
    if a is None:
        return dict(b)
    out = dict(a)
    for r, (y, ld) in b.items():
        if r not in out or y < out[r][0]:
            out[r] = (y, ld)
    return out


def _key(st):
    return frozenset((r, y) for r, (y, _) in st.items())


def check(body, max_states=64):
    """Path-sensitive where affordable: every distinct in-flight state reaching
    a block is propagated on its own (the ring state at a point is almost always
    the same whatever the path, so this stays small); a block reached in more
    than `max_states` states falls back to the merged (union, min-count) state."""
    problems = set()
    if re.search(r"s_set_gpr_idx_on|v_movrel|scratch_|buffer_store_dword .*off, s\[0:3\]", body):
        problems.add("dynamic GPR indexing or scratch access")
    blocks = _blocks(body)
    index = {nm: i for i, (nm, _, _) in enumerate(blocks)}
    seen = [dict() for _ in blocks]  # block -> {state key: state}
    merged = [None] * len(blocks)
    work = [(0, {})]
    while work:
        i, st0 = work.pop()
        k = _key(st0)
        if len(seen[i]) >= max_states:
            m = _merge(merged[i], st0)
            if merged[i] is not None and _key(m) == _key(merged[i]):
                continue
            merged[i] = m
            st0 = m
        elif k in seen[i]:
            continue
        else:
            seen[i][k] = st0
            merged[i] = _merge(merged[i], st0)
        nm, ins, succ = blocks[i]
        st = dict(st0)
        for t in ins:
            st = _step(st, t, problems, nm)
        for sname in succ:
            j = index.get(sname)
            if j is not None:
                work.append((j, st))
    return sorted(problems)


if __name__ == "__main__":
    # asm_ring_check.py FILE.s [SUBSTR]                  full dataflow check of the matching kernels
    # asm_ring_check.py FILE.s --pinned SUBSTR FIRST LAST  pinned-ring check (the build runs this on
    #                                                      the product gv4 / log-stream objects)
    text = open(sys.argv[1]).read()
    pinned = len(sys.argv) > 2 and sys.argv[2] == "--pinned"
    sub = sys.argv[3] if pinned else (sys.argv[2] if len(sys.argv) > 2 else "")
    bad = seen = 0
    for sym, body in kernels(text).items():
        if sub in sym:
            seen += 1
            p = check_pinned(body, int(sys.argv[4]), int(sys.argv[5])) + check_local(body) if pinned else check(body)
            bad += len(p)
            for x in p[:8]:
                print(sym[:60], x[:240])
    if pinned and not seen:
        print("no kernel matches", sub)
        bad = 1
    print("problems", bad)
    sys.exit(1 if bad else 0)
