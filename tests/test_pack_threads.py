"""The dataset packing (sk_api.cpp pack_dataset) runs its per-example passes
on host threads and appends at prefix offsets: the packed arrays must not
depend on the thread count.  tools/pack_compare.cpp includes the library
source and hashes every packed array (the y-role records, every SK_BIG x-role
array, the per-example ex_* vectors and key tables); it is built here (host
code only) and run with one thread and with eight (SK_PACK_THREADS), and both
must equal GOLDEN: the hashes of the serial packer before the threaded one
(commit 61ba1f6^, built in a worktree with this pack_compare.cpp, r05), so a
rebase bug that does not depend on the thread count fails here too."""
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


GOLDEN = {(300, 150): ("36d6bd2e8250904e", "287b3489cc46be35"),
          (64, 300): ("88c43b92757d6d0c", "7683c19231feea38"),
          (7, 40): ("5103f9f17bc7fe14", "f110ddedec494801")}


@pytest.mark.parametrize("n,L", sorted(GOLDEN))
def test_packing_independent_of_threads(pack_compare, n, L):
    for t in ("1", "8"):
        r = subprocess.run([pack_compare, str(n), str(L)], env=dict(os.environ, SK_PACK_THREADS=t),
                           capture_output=True, text=True, timeout=300, check=True)
        line = r.stdout.strip().splitlines()[-1]
        assert line.startswith("rc=0"), line
        hy = line.split("y-hash ")[1].split()[0]
        hx = line.split("x-hash ")[1].split()[0]
        assert (hy, hx) == GOLDEN[(n, L)], (t, hy, hx)
