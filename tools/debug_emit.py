#!/usr/bin/env python3
"""Diagnoses jl_log_emit_dev against the oracle LogWriter: per-fragment header
and payload comparison, plus the same fragments through jl_crc32c_batch_dev
(MODE_CRC with init = typeCrc[t]) to separate the header mode from the stream
kernel's CRC."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import jleveldb_amd as jl  # noqa: E402
from oracle import oracle  # noqa: E402

torch.cuda.set_device(0)
jl.init(0)
dev = torch.device("cuda:0")
rng = np.random.default_rng(40)
lens = rng.choice([0, 1, 6, 7, 100, 1056, 32761, 32762, 40000, 100000], size=80).astype(np.uint32)
payloads = [rng.integers(0, 256, int(k), dtype=np.uint8).tobytes() for k in lens]
offs = np.zeros(lens.size, np.uint64)
offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
src = np.frombuffer(b"".join(payloads), dtype=np.uint8)
plan = jl.log_layout(offs, lens, 0)
got = jl.log_emit_dev(torch.from_numpy(src.copy()).to(dev), plan).cpu().numpy()
ref = np.frombuffer(oracle.log_write(payloads, 0), dtype=np.uint8)
print("bytes equal:", np.array_equal(got, ref), "n_frags", plan["len"].size)
typecrc = [jl.Crc32C.value(bytes([t])) for t in range(5)]
bad = 0
for i, (h, n, t) in enumerate(zip(plan["hdr_off"], plan["len"], plan["type"])):
    h, n = int(h), int(n)
    hd_ok = np.array_equal(got[h:h + 7], ref[h:h + 7])
    pl_ok = np.array_equal(got[h + 7:h + 7 + n], ref[h + 7:h + 7 + n])
    if not (hd_ok and pl_ok):
        bad += 1
        K = (n + 255) // 256
        f = 256 * K - n
        print(f"frag {i}: hdr {h} len {n} type {t} ptr&3 {(h + 7) & 3} K {K} f {f} l0 {f >> 2} r {f & 3} "
              f"header_ok {hd_ok} payload_ok {pl_ok}")
print("bad fragments:", bad)
# the same ranges through MODE_CRC with per-fragment init = typeCrc[t]
log_d = torch.from_numpy(ref.copy()).to(dev)
po = (plan["hdr_off"] + 7).astype(np.uint64)
init = np.array([typecrc[t] for t in plan["type"]], np.uint32)
crc = jl.crc32c_batch_dev(log_d, torch.from_numpy(po.view(np.int64)).to(dev),
                          torch.from_numpy(plan["len"].view(np.int32)).to(dev),
                          init=torch.from_numpy(init.view(np.int32)).to(dev)).cpu().numpy().view(np.uint32)
want = np.array([int.from_bytes(ref[int(h):int(h) + 4].tobytes(), "little") for h in plan["hdr_off"]], np.uint32)
print("MODE_CRC with init: mismatches", np.nonzero(crc != want)[0][:20])

# (a) MODE_CRC over the kernel-written image itself
got_d = jl.log_emit_dev(torch.from_numpy(src.copy()).to(dev), plan)
crc2 = jl.crc32c_batch_dev(got_d, torch.from_numpy(po.view(np.int64)).to(dev),
                           torch.from_numpy(plan["len"].view(np.int32)).to(dev),
                           init=torch.from_numpy(init.view(np.int32)).to(dev)).cpu().numpy().view(np.uint32)
print("(a) MODE_CRC over emitted image: mismatches", np.nonzero(crc2 != want)[0][:20])
# (b) bounds-checked debug variant (all loads through VGPR addresses)
os.environ["JL_STREAM_DEBUG"] = "0:ffffffffffffffff"
g = jl.log_emit_dev(torch.from_numpy(src.copy()).to(dev), plan).cpu().numpy()
print("(b) debug variant emit equal:", np.array_equal(g, ref))
del os.environ["JL_STREAM_DEBUG"]
# (c) r1 chunked kernel
os.environ["JL_GENERAL"] = "chunk"
g = jl.log_emit_dev(torch.from_numpy(src.copy()).to(dev), plan).cpu().numpy()
print("(c) chunk kernel emit equal:", np.array_equal(g, ref))
del os.environ["JL_GENERAL"]
# (d) stream kernel again, depth 16 and 48
for dpt in ("16", "48"):
    os.environ["JL_STREAM_DEPTH"] = dpt
    g = jl.log_emit_dev(torch.from_numpy(src.copy()).to(dev), plan).cpu().numpy()
    print(f"(d) depth {dpt} emit equal:", np.array_equal(g, ref))
