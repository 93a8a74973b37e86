"""CPU sanitizer runs (SURVEY §5 "sanitizers"): the ToMe oracle
(oracle/tome_ref.c) under ASan + UBSan, and the host half of libmmt_hip's ToMe / pruning / core
C-ABI dispatch under ASan, both built by tests/asan/build_asan.sh into a temporary directory (the
address sanitizer on host code only; nothing here launches a kernel or needs a GPU). Each driver
prints OK after its checks; any out-of-bounds access, use-after-free or undefined behaviour aborts
it with a sanitizer report instead."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

HERE = Path(__file__).resolve().parent


@pytest.fixture(scope="module")
def asan_dir(tmp_path_factory):
    if not (shutil.which("gcc") and Path(os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")).exists()):
        pytest.skip("gcc / hipcc not available")
    out = tmp_path_factory.mktemp("mmt_asan")
    r = subprocess.run(["bash", str(HERE / "asan" / "build_asan.sh"), str(out)], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    return out


def _run(exe, leaks):
    env = dict(os.environ, ASAN_OPTIONS=f"detect_leaks={int(leaks)}:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout[-4000:] + r.stderr[-4000:]


def test_tome_oracle_under_asan_ubsan(asan_dir):
    _run(asan_dir / "tome_ref_asan", leaks=True)


def test_abi_host_dispatch_under_asan(asan_dir):
    # the HIP runtime's own allocations are not this library's: leak checking off
    _run(asan_dir / "abi_host_asan", leaks=False)
