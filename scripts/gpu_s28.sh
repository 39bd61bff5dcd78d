set -o pipefail
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 400 python scripts/op_census_maskrcnn.py --batch 1 > gpurun_out/op_census28.txt 2> gpurun_out/op_census28.err || exit 1
