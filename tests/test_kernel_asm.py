"""Static checks of the product HIP kernels' ISA (CPU; hipcc cross-compiles gfx950 here).

The bf16 noise-MLP kernel (csrc/noise_mlp.hip solo::) reads its weight fragments and biases with
inline-asm ds_reads and counted lgkmcnt waits.  The compiler sees an asm read's output as written
at once, so if it ever reused, copied or spilled such a register before the wait that covers it,
data landing later would corrupt the register (a round-5 development build clobbered a 64-bit
address that way and faulted the GPU).  tools/asm_hazard.py scans the built ISA for any use of a
register with an LDS read in flight."""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="hipcc not installed")
@pytest.mark.parametrize("kernel", ["noise_mlp_solo_kernel"])
def test_no_register_use_while_an_lds_read_is_in_flight(kernel):
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "asm_hazard.py"), kernel],
                       capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 hazard(s)" in r.stdout
