# Host C API tests + reference-shape per-call timings (gpurun).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_native_capi.py tests/test_convolve.py tests/test_conv_paths.py tests/test_matrix.py tests/test_arithmetic.py tests/test_mathfun.py tests/test_wavelet.py tests/test_normalize.py tests/test_detect_peaks.py tests/test_memory.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_hostapi.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_hostapi.log
if [ $rc -ne 0 ] || grep -q '+++ Timeout +++' gpurun_out/pytest_hostapi.log; then echo "failed/hung: stop"; exit 1; fi
timeout -k 10 600 python -u tools/bench_reference_shapes.py run > gpurun_out/refshapes.log 2>&1; tail -4 gpurun_out/refshapes.log
