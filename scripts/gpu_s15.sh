set -o pipefail
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke15.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --model gpt3-6.7b --micro-batch-size 2 --steps 5 --warmup 2 --no-maskrcnn > gpurun_out/bench15_gpt3.log 2>&1
