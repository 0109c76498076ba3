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


def test_production_library_holds_only_launched_kernel_forms():
    """Measured-and-rejected kernel variants are not compiled into the
    production .so (round 5): one compile-time row / column kernel per plan
    of PHD_CT_ROWS / PHD_CT_COLS (columns: and its prefetch form), K1's two-block and one-block forms only (x
    the small-grid mask form), one statistics kernel."""
    import subprocess
    so = os.path.join(ROOT, "photohive_dsp_amd", "PhotoHive_DSP_lib", "libreport_data.so")
    out = subprocess.run(["nm", "-C", so], capture_output=True, text=True, check=True).stdout
    stubs = re.findall(r"__device_stub__(\w+)", out)
    count = {k: stubs.count(k) for k in set(stubs)}
    with open(os.path.join(ROOT, "photohive_dsp_amd", "csrc", "phd_internal.h")) as f:
        src = f.read()

    def plans(name):
        n = 0
        for ln in src[src.index(f"#define {name}(X)"):].split("\n")[1:]:
            n += ln.strip().startswith("X(")
            if not ln.rstrip().endswith("\\"):
                break
        return n

    assert count.get("k_rows_ct") == plans("PHD_CT_ROWS"), count
    # columns: the plain form per plan, plus the prefetch form where it fits
    assert plans("PHD_CT_COLS") < count.get("k_cols_ct", 0) <= 2 * plans("PHD_CT_COLS"), count
    assert count.get("k_k1t") == 6, count          # <512, tri> and <1024, tri / full>, x SMALL
    assert count.get("k_rgb_stats") == 1, count


def test_import_leaves_environment_alone():
    """Importing the package changes no process-wide setting (VERDICT r5 item
    7): GPU_MAX_HW_QUEUES stays unset until the caller opts in with
    configure_hw_queues(), which never overrides a value already chosen."""
    import subprocess
    import sys
    code = ("import os, json; before = dict(os.environ); import photohive_dsp_amd as p; "
            "after = dict(os.environ); changed = sorted(k for k in set(before) | set(after) "
            "if before.get(k) != after.get(k)); "
            "w1 = p.configure_hw_queues(8); v1 = os.environ.get('GPU_MAX_HW_QUEUES'); "
            "w2 = p.configure_hw_queues(4); v2 = os.environ.get('GPU_MAX_HW_QUEUES'); "
            "print(json.dumps([changed, w1, v1, w2, v2]))")
    env = {k: v for k, v in os.environ.items() if k != "GPU_MAX_HW_QUEUES"}
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    import json
    changed, w1, v1, w2, v2 = json.loads(r.stdout.strip().splitlines()[-1])
    assert changed == [], changed
    assert (w1, v1, w2, v2) == (True, "8", False, "8")
