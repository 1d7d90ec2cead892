# multi-rank rehearsal of the bench's N > 1 path on ONE GPU over gloo (the driver runs the real N = 2..8 over RCCL):
# dp + row-shard at 2 and 4 ranks, small steps; then the one-rank sharded path over RCCL
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for N in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
      --master-port $((29600 + N)) bench.py --gpus $N --steps 3 --warmup 1 --cpu-baseline 0 --legs none --backend gloo \
      > gpurun_out/dist_$N.json 2> gpurun_out/dist_$N.err || exit $?
  python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], r['value'], r['ms_per_step'], r['config']['parallelism'])" gpurun_out/dist_$N.json $N
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --legs none --sharded > gpurun_out/dist_s1.json 2> gpurun_out/dist_s1.err || exit $?
python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('sharded1', r['value'], r['ms_per_step'], r['config']['parallelism'])" gpurun_out/dist_s1.json
