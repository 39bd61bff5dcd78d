# final validation of the session: smoke, full GPU test suite, default bench (GPT + Mask R-CNN)
set -o pipefail
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final2_smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final2_tests.log 2>&1 || exit 1
timeout -k 10 500 python bench.py > gpurun_out/final2_bench.log 2>&1 || exit 1
