"""The built library carries no wide-store data hazard: no buffer/global store of
more than 8 bytes is followed, with zero wait states, by an instruction that writes the VGPRs
holding its data.  The compiler pads its own instructions; this catches inline asm that lands
behind such a store (the cause of the round-4 RGB warp's intermittent wrong pixels).  Runs on
the CPU over the gfx950 code objects inside libkcmc.so (llvm-objdump)."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "keypoint-consensus-motion-correction_amd", "libkcmc.so")
SCAN = os.path.join(REPO, "tools", "debug", "store_hazard_scan.py")


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                    reason="needs the built libkcmc.so and ROCm's llvm-objdump")
def test_no_wide_store_data_hazard_in_the_library():
    r = subprocess.run([sys.executable, SCAN, LIB], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    n_wide = int(r.stdout.strip().splitlines()[-1].split()[0])
    assert n_wide > 100  # the scan saw the warp's wide stores (the RGB / RGBA paths and the rest)


def test_scanner_flags_the_round4_pattern():
    sys.path.insert(0, os.path.dirname(SCAN))
    import store_hazard_scan as S

    bad = ("0000000000001000 <k>:\n"
           "\tbuffer_store_dwordx3 v[6:8], v4, s[12:15], s3 offen nt // 000000001000: E07C1000 80030604\n"
           "\tv_bfe_u32 v6, v3, 11, 5                                // 000000001008: D1C80006 022D1703\n")
    ok = bad.replace("\tv_bfe_u32 v6", "\ts_nop 0\n\tv_bfe_u32 v6")
    assert len(S.scan_text(bad)) == 1 and S.scan_text(ok) == []
    g = ("0000000000002000 <g>:\n\tglobal_store_dwordx4 v[2:3], v[4:7], off\n\tv_mov_b32_e32 v5, 0\n"
         "\tglobal_store_dwordx4 v[2:3], v[4:7], off\n\tv_mov_b32_e32 v2, 0\n")
    assert [f[2] for f in S.scan_text(g)] == ["v_mov_b32_e32 v5, 0"]  # data, not the address, counts
