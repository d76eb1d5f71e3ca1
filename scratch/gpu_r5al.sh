set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_native_resnet_model.py -m gpu -q -k aux_stream --timeout 120 --timeout-method thread > gpurun_out/r5al_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r5al_tests.log
