#!/usr/bin/env python3
"""Regenerates the pinned ring-slot table of general_v4.hip for ring depth P
(slots in v[256-4P .. 255], compiler budget 256-4P) and the matching range of
tools/asm_ring_check.check_pinned.  Usage: python tools/gv4_slots.py P"""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = int(sys.argv[1])
base = 256 - 4 * P
p = os.path.join(ROOT, "jleveldb_amd", "csrc", "general_v4.hip")
s = open(p).read()
a = s.index("#define JL_GV4_SLOTS(X) \\\n")
b = s.index("\n\n", a)
slots = "\n".join(f'    X({u}, "v[{base + 4 * u}:{base + 3 + 4 * u}]", "v{base + 4 * u}", "v{base + 1 + 4 * u}", '
                  f'"v{base + 2 + 4 * u}", "v{base + 3 + 4 * u}")' + (" \\" if u < P - 1 else "") for u in range(P))
s = s[:a] + "#define JL_GV4_SLOTS(X) \\\n" + slots + s[b:]
s = re.sub(r"// the \d+ ring slots: \(slot, register quad, its 4 registers\), pinned in v\d+..v255\n"
           r"#define JL_GV4_RING \d+\n#define JL_GV4_VGPR_BUDGET \d+",
           f"// the {P} ring slots: (slot, register quad, its 4 registers), pinned in v{base}..v255\n"
           f"#define JL_GV4_RING {P}\n#define JL_GV4_VGPR_BUDGET {base}", s)
assert P <= 22, "the allocator cap (JL_GV4_WAVES_PER_EU 3 = 168 VGPRs) must stay below the pinned ring"
open(p, "w").write(s)
c = os.path.join(ROOT, "tools", "asm_ring_check.py")
t = open(c).read()
t = re.sub(r"def check_pinned\(body, first=\d+, last=255\):", f"def check_pinned(body, first={base}, last=255):", t)
open(c, "w").write(t)
print("ring", P, "pinned from", base)
