export TMPDIR=/tmp
mkdir -p gpurun_out/r5f
Q="--consolidate-steps 0 --sharded-steps 0 --routed-steps 0 --global-batch 0"
for i in 1 2 3; do
  timeout -k 10 300 python bench.py $Q > gpurun_out/r5f/h$i.json 2> gpurun_out/r5f/h$i.err || exit 1
done
