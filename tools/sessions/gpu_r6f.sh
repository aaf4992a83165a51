#!/bin/bash
# round 6 (lab library shipped): C3 encode layouts with the plane mask (tools/probe_c3_planes.py)
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/r6f
export TMPDIR=/tmp
NUMCODECS_AMD_LIB=tools/_build/libmcodec_lab.so timeout -k 10 240 python3 tools/probe_c3_planes.py > gpurun_out/r6f/probe_c3_planes.json 2> gpurun_out/r6f/probe.err || { tail gpurun_out/r6f/probe.err; exit 1; }
cat gpurun_out/r6f/probe_c3_planes.json
