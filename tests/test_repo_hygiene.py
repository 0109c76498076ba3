"""Repository contracts that are not numerics: the reference's compiled
sources stay off the GPU box, and the product library
reads only the environment switches its tests name."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ignore_patterns():
    with open(os.path.join(ROOT, ".gpurunignore")) as f:
        return [ln.strip() for ln in f if ln.strip() and not ln.startswith("#")]


def test_gpurunignore_excludes_reference_builds():
    """Every directory oracle/Makefile writes from REF_SRC (the reference's
    own C compiled where it lies) or from the sanitizer build is excluded from
    the gpurun snapshot."""
    with open(os.path.join(ROOT, "oracle", "Makefile")) as f:
        mk = f.read()
    outdirs = set(re.findall(r"\$\(HERE\)(_\w+)/", mk))
    assert {"_ref", "_san"} <= outdirs, outdirs
    pats = _ignore_patterns()
    for d in sorted(outdirs):
        assert f"./oracle/{d}" in pats or f"oracle/{d}" in pats, f"oracle/{d} travels to the GPU box"


def test_production_library_reads_few_environment_switches():
    """The production .so reads only PHD_VERBOSE, PHD_QUIET and PHD_LANES from
    the environment; the timing experiments' switches go through phd_knob,
    which only the ablate build compiles to getenv (phd_internal.h)."""
    csrc = os.path.join(ROOT, "photohive_dsp_amd", "csrc")
    names = set()
    for fn in os.listdir(csrc):
        if fn.endswith((".hip", ".cpp", ".h")):
            with open(os.path.join(csrc, fn)) as f:
                names.update(re.findall(r'\bgetenv\("(\w+)"\)', f.read()))
    assert names <= {"PHD_VERBOSE", "PHD_QUIET", "PHD_LANES"}, sorted(names)
    with open(os.path.join(csrc, "phd_internal.h")) as f:
        src = f.read()
    knob = src[src.index("inline const char* phd_knob"):]
    knob = knob[:knob.index("\n}\n")]
    assert "#ifdef PHD_ABLATE_BUILD" in knob and "return nullptr;" in knob
