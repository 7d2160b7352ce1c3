"""Build-time guard for the hand-pipelined loads (CPU only, no GPU).

Every engine kernel issues its HBM loads as inline asm and waits for them with
hand-counted s_waitcnt vmcnt(N).  If the compiler copies a ring register
between the asm load and its wait (dynamic indexing of a rolled loop, a spill,
a register-allocation copy) the kernel silently reads stale data — r1 hit
exactly this (s_set_gpr_idx copies in a rolled ring loop).  This compiles every
kernel translation unit to gfx950 assembly and rejects any such pattern
(tools/asm_ring_check.py)."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "jleveldb_amd", "csrc")
UNITS = ([("jlcrc_kernels.hip", []), ("fixed_v4.hip", [])] + [("stream_kernel.hip", [f"-DJL_MODE={m}"]) for m in range(5)]
         + [("general_v4.hip", [f"-DJL_MODE={m}"]) for m in (0, 1, 2, 5)] + [("log_stream.hip", []),
                                                                              ("log_chunks.hip", [])])


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    d = tmp_path_factory.mktemp("asm")

    def one(i):
        src, defs = UNITS[i]
        out = d / f"u{i}.s"
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-Wno-pass-failed",
                        "--cuda-device-only", "-S", *defs, "-o", str(out), os.path.join(CSRC, src)],
                       check=True, capture_output=True)
        return out.read_text()

    with ThreadPoolExecutor(max_workers=min(6, os.cpu_count() or 1)) as ex:
        return "\n".join(ex.map(one, range(len(UNITS))))


def test_no_stale_ring_reads(asm):
    """Straight-line ring kernels (the 4 KiB kernels) get the full control-flow
    dataflow check; the general v4 kernel, whose ring is pinned in v192..v255,
    the check that no compiler code touches those registers; the stream and r1
    chunk kernels the block-local one (their CFGs carry SGPR-correlated
    branches that make the path analysis report infeasible paths; their GPU
    parity tests cover them)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from asm_ring_check import check, check_local, check_pinned, kernels

    ks = {s: b for s, b in kernels(asm).items() if "crc_" in s}
    assert sum("crc_stream_kernel" in s for s in ks) >= 15
    assert any("crc_fixed4k_v4" in s for s in ks)
    assert sum("crc_gv4_kernel" in s for s in ks) >= 4
    assert any("crc_logstream_kernel" in s for s in ks)
    branchy = ("crc_stream_kernel",)

    def one(s, b):
        if "crc_gv4_kernel" in s:
            return check_pinned(b, first=88, last=127) + check_local(b)  # 1024 threads: v88..v127
        if "crc_logstream_kernel" in s:  # ring pinned in v136..v167 (12 waves per CU)
            return check_pinned(b, first=136, last=167) + check_local(b)
        return check_local(b) if any(k in s for k in branchy) else check(b)

    problems = {s: one(s, b) for s, b in ks.items()}
    assert not {s: p[:3] for s, p in problems.items() if p}


def _sgprs(tok):
    import re

    m = re.fullmatch(r"s\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"s(\d+)", tok)
    return {int(m.group(1))} if m else set()


def test_no_smem_address_clobbered_inside_an_asm_block(asm):
    """Inside one inline-asm block, a scalar load's destination must not overlap
    the address SGPRs of a later scalar load of the same block: the first load's
    data can land before the second one reads its address (r1: the round
    descriptors' two s_load_dwordx16 shared s[16:17] / s[16:31]; a descheduled
    wave then loaded from a descriptor word, an aperture-violation fault)."""
    bad = []
    block = None
    for line in asm.split("\n"):
        if ";;#ASMSTART" in line:
            block = []
            continue
        if ";;#ASMEND" in line:
            block = None
            continue
        if block is None:
            continue
        ins = line.split(";")[0].strip()
        if not ins.startswith("s_load") and not ins.startswith("s_buffer_load"):
            continue
        ops = [o.strip() for o in ins.split(None, 1)[1].split(",")]
        dst, addr = _sgprs(ops[0]), _sgprs(ops[1])
        if any(addr & d for d in block):
            bad.append(ins)
        block.append(dst)
    assert not bad, bad[:5]


def test_no_scratch_memory(asm):
    """No kernel keeps anything in scratch (private) memory: r3's lc_dense had its
    prefetched block bytes (an array of HIP uint4) placed there by the compiler,
    so every byte was written to memory and read back (PMC WRITE_SIZE 4.4 GB per
    4 GiB log)."""
    import re

    sizes = re.findall(r"\.name:\s+(\S+)\n(?:.*\n)*?\s+\.private_segment_fixed_size:\s+(\d+)", asm)
    assert len(sizes) >= 30
    assert not [(n, int(z)) for n, z in sizes if int(z)], [(n, int(z)) for n, z in sizes if int(z)][:5]
