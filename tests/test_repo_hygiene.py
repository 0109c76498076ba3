"""Repository contracts that are not numerics: the product library reads only
the environment switches its documentation names (the reference builds'
absence from the GPU box is test_abi.py's)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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
