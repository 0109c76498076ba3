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
