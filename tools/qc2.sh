set -e
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 300 python tools/quickcheck.py > gpurun_out/qc_filter.log 2>&1
RTW_FILTER=0 timeout -k 10 300 python tools/quickcheck.py > gpurun_out/qc_nofilter.log 2>&1
