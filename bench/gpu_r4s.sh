set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
H="--consolidate-steps 0 --sharded-steps 0 --no-persistent-graph --routed-steps 0 --global-batch 0 --recall-queries 256 --steps 30"
nproc > gpurun_out/hs_env.txt; cat /sys/fs/cgroup/cpu.max >> gpurun_out/hs_env.txt 2>/dev/null; uptime >> gpurun_out/hs_env.txt
LZK_PROF_HEADLINE=1 timeout -k 10 300 python -u bench.py $H --json-out gpurun_out/hs_p.json > gpurun_out/hs_p.log 2> gpurun_out/hs_p.err || exit 2
