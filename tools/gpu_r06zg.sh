# round 6, call zg: the whole -m gpu suite against the checked build (libavse_debug.so: device-side protocol / bounds
# checks) on the final kernels
set -o pipefail
mkdir -p gpurun_out
AVSE_LIBRARY=$(pwd)/audio-visual-speech-enhancement_amd/libavse_debug.so timeout -k 10 1100 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r06zg_checked_suite.log 2>&1
rc=$?
tail -5 gpurun_out/r06zg_checked_suite.log
exit $rc
