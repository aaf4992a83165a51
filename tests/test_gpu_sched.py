"""The product library's schedule is fixed (numcodecs_amd/csrc/mc_sched.h:
no environment variable is read).  Every alternative schedule the lab
library can select (tools/lab/lab_sched.hip) is checked against the oracle
here, in ONE child process that runs the public codecs on top of the lab
library (tests/sched_check.py), so a measured-and-rejected setting stays
correct if a later sweep picks it."""

import json
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LAB = os.path.join(ROOT, "tools", "_build", "libmcodec_lab.so")


@pytest.mark.gpu
def test_every_lab_schedule_matches_the_oracle(device):
    from tests.helpers import check_lab_build

    check_lab_build()
    if not os.path.exists(LAB):
        pytest.skip("lab library not built (make -C tools/lab)")
    env = {k: v for k, v in os.environ.items() if not k.startswith("MCODEC_")}
    env["NUMCODECS_AMD_LIB"] = LAB
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "sched_check.py")], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    bad = [c for c in d["cases"] if not c["ok"]]
    assert not bad, bad
    fields = {c["field"] for c in d["cases"]}
    # every field of mc_sched_t (numcodecs_amd/csrc/mc_sched.h) is walked
    with open(os.path.join(ROOT, "numcodecs_amd", "csrc", "mc_sched.h")) as f:
        declared = set(re.findall(r"^\s+int (\w+);", f.read(), re.M))
    assert fields == declared and all(sum(1 for c in d["cases"] if c["field"] == f and not c["default"]) >= 1
                                     for f in fields)


def test_product_library_reads_no_environment():
    """No getenv in the product sources, and the product .so imports none."""
    csrc = os.path.join(ROOT, "numcodecs_amd", "csrc")
    for f in os.listdir(csrc):
        if f.endswith((".hip", ".h")):
            with open(os.path.join(csrc, f)) as fh:
                assert "getenv" not in fh.read(), f
    so = os.path.join(ROOT, "numcodecs_amd", "_lib", "libmcodec.so")
    if os.path.exists(so):
        r = subprocess.run(["nm", "-D", "--undefined-only", so], capture_output=True, text=True)
        if r.returncode == 0:
            assert not any(ln.split()[-1].startswith(("getenv", "secure_getenv")) for ln in r.stdout.splitlines()
                           if ln.strip())
