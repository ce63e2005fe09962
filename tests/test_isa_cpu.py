"""Static ISA checks of the shipped LDS-DMA kernels (no GPU): every global_load_lds
takes its LDS base from an M0 write in its own basic block with no other M0 write
and no scratch (spill) access in between, and no kernel that issues LDS-DMA loads
spills.  Round 2's 4-waves/SIMD 8-plane-spool variant of k_env_step_bits128, which
faulted on the box, is the one build known to break the second and third rules
(tools/isa_lds_dma_check.py)."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_lds_dma_m0_windows_and_no_spills(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "isa_lds_dma_check.py")],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    n = int(r.stdout.strip().splitlines()[-1].split()[0])
    assert n >= 100, r.stdout[-500:]          # the bit-sliced kernels' DMA loads were seen
