set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_delta_walk.py tests/test_gpu_delta_spec.py tests/test_gpu_delta_spec2.py tests/test_gpu_delta.py tests/test_gpu_codecs.py tests/test_gpu_next.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/walk_tests.log 2>&1
rc=$?; tail -4 gpurun_out/walk_tests.log; echo "tests rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python -u tools/probe_fspec_walk.py f4 ${PROBE_MIB:-16} ${PROBE_MODE:-quick} > gpurun_out/probe_walk_f4.json 2> gpurun_out/probe_walk_f4.err
rc=$?; grep -v amdgpu.ids gpurun_out/probe_walk_f4.err | tail -14; echo "probe rc=$rc"
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 200 python -u tools/probe_verify_overhead.py > gpurun_out/probe_verify_overhead.json 2>&1
rc=$?; tail -1 gpurun_out/probe_verify_overhead.json; echo "verify rc=$rc"
