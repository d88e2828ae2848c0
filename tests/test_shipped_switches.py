"""The shipped library carries no wrong-value switches: the cost experiments
that skipped work (SK_STR_SKIP, SK_SKIP_LOOPS, SK_PHI_EXP, SK_ROW_EXP) and the
variants measured slower and dropped (SK_SWEEP_GAP, SK4C_P2P, SK4C_RANGE,
SK4P_RANGE) are gone from the default sources, and every run-time knob (a
getenv, or an SK_KNOB of the experiments build) is one INTEGRATION.md lists
(each selects a schedule, a kernel variant of equal results, or a
diagnostic).  tests/test_explib.py checks that the shipped library reads none
but the diagnostics and the thread count."""
import pathlib
import re

ROOT = pathlib.Path(__file__).resolve().parents[1]
CSRC = ROOT / "stem_kernel_amd" / "csrc"
REMOVED = ["SK_STR_SKIP", "SK_SKIP_LOOPS", "SK_PHI_EXP", "SK_ROW_EXP", "SK_SWEEP_GAP", "SK4C_P2P",
           "SK4C_RANGE", "SK4P_RANGE"]


def _sources():
    return [p for p in CSRC.rglob("*") if p.suffix in (".cpp", ".hip", ".h", ".hpp", ".inc")] + \
        list((ROOT / "include").rglob("*.h*"))


def test_removed_switches_absent():
    hits = [(p.name, sw) for p in _sources() for sw in REMOVED if sw in p.read_text()]
    assert not hits, hits


def test_runtime_knobs_documented():
    knobs = set()
    for p in _sources():
        knobs |= set(re.findall(r'(?:getenv|SK_KNOB)\("([A-Z0-9_]+)"\)', p.read_text()))
    doc = (ROOT / "INTEGRATION.md").read_text()
    missing = sorted(k for k in knobs if f"`{k}`" not in doc)
    assert not missing, f"run-time knobs not listed in INTEGRATION.md: {missing}"
