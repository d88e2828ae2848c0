"""The dataset packing (sk_api.cpp pack_dataset) runs its per-example passes
on host threads and appends at prefix offsets: the packed arrays must not
depend on the thread count.  tools/pack_compare.cpp includes the library
source and hashes every packed array; it is built here (host code only) and
run with one thread and with eight (SK_PACK_THREADS)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def pack_compare(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("pc") / "pack_compare")
    src = os.path.join(ROOT, "stem_kernel_amd", "csrc", "sk_api.cpp")
    lib = os.path.join(ROOT, "stem_kernel_amd")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "include"), "-I",
                    os.path.join(ROOT, "stem_kernel_amd", "csrc"), "-D__HIP_PLATFORM_AMD__", f'-DSRC="{src}"',
                    os.path.join(ROOT, "tools", "pack_compare.cpp"), "-o", exe, "-L", lib, "-lstem_kernel_amd",
                    f"-Wl,-rpath,{lib}", "-L/opt/rocm/lib", "-lrccl"], check=True, timeout=600)
    return exe


@pytest.mark.parametrize("n,L", [(300, 150), (64, 300), (7, 40)])
def test_packing_independent_of_threads(pack_compare, n, L):
    out = {}
    for t in ("1", "8"):
        r = subprocess.run([pack_compare, str(n), str(L)], env=dict(os.environ, SK_PACK_THREADS=t),
                           capture_output=True, text=True, timeout=300, check=True)
        line = r.stdout.strip().splitlines()[-1]
        assert line.startswith("rc=0"), line
        out[t] = line.split("y-hash")[1]
    assert out["1"] == out["8"]
