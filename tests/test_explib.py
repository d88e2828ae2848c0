"""The kernel-variant comparisons (tests marked `explib`: four-state vs K-sum
vs column 4-D planes, Gamma / Phi schedules on and off, the forced big-y
kernel, general vs fast string and BPLA kernels, BPLA chunking, 4-D stream
parts) need switches the shipped library does not read (DESIGN.md §4,
INTEGRATION.md "Run-time knobs").  The experiments build
(build/libstem_kernel_amd_exp.so: the same sources with -DSK_EXPERIMENTS,
`make exp`) reads them; these tests run it in ONE child pytest process (the
library is loaded once per process) and require every variant test to pass.
On the CPU the shipped library is checked to carry no switch at all."""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIPPED = os.path.join(ROOT, "stem_kernel_amd", "libstem_kernel_amd.so")
EXP = os.path.join(ROOT, "build", "libstem_kernel_amd_exp.so")
# the only environment variables the shipped library may read: diagnostics
# and the host packing thread count
ALLOWED = {"SK_HOST_STATS", "SK_PACK_STATS", "SK_PHI_STATS", "SK_PACK_THREADS"}


def _sk_strings(path):
    data = open(path, "rb").read()
    return {m.decode() for m in re.findall(rb"(?<![A-Za-z0-9_])(SK4?C?_[A-Z0-9_]{2,})\x00", data)}


def test_shipped_library_reads_no_switches():
    names = _sk_strings(SHIPPED)
    assert names <= ALLOWED, sorted(names - ALLOWED)
    from stem_kernel_amd._lib import lib
    if os.path.realpath(os.environ.get("SK_LIB_PATH") or SHIPPED) == os.path.realpath(SHIPPED):
        assert lib().sk_experiments() == 0


def test_experiments_build_has_the_switches():
    names = _sk_strings(EXP)
    for k in ("SK4_NO_GSUM", "SK4_SPAN", "SK_NO_GAMMA", "SK_STR_GENERAL", "SK_BPLA_GENERAL", "SK_FORCE_BIG_Y"):
        assert k in names, k


@pytest.mark.gpu
def test_kernel_variants_on_experiments_build():
    env = dict(os.environ, SK_LIB_PATH=EXP, PYTHONUNBUFFERED="1")
    cmd = [sys.executable, "-u", "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "--timeout", "300",
           "--timeout-method", "thread", "-m", "gpu and explib", os.path.join(ROOT, "tests")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=1500)
    tail = "\n".join((r.stdout + r.stderr).strip().splitlines()[-25:])
    assert r.returncode == 0, tail
    m = re.search(r"(\d+) passed", r.stdout)
    assert m and int(m.group(1)) >= 10 and "skipped" not in r.stdout.splitlines()[-1], tail
    print(tail.splitlines()[-1])
