# Multi-rank rehearsal on ONE GPU over gloo (RCCL refuses several ranks per device):
# bench.py at world size 4 (cdssm) and 2 (mlp, bert, chunked) — the driver's torchrun contract.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PAGEVEC_DIST_BACKEND=gloo
run() {  # name nproc args...
  local name=$1 np=$2; shift 2
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 1000)) bench.py --gpus $np "$@" > gpurun_out/rehearse_$name.log 2>&1
  local rc=$?; echo "$name rc=$rc $(grep '^{' gpurun_out/rehearse_$name.log | tail -1 | cut -c1-200)"; return $rc
}
run cdssm4 4 --steps 3 --warmup 2 --batch 512 --quality-steps 0 --recall 256 &&
run mlp2 2 --model mlp --steps 3 --warmup 2 --batch 512 --quality-steps 0 --recall 256 &&
run bert2 2 --model bert --steps 2 --warmup 2 --batch 32 --quality-steps 0 --recall 64 &&
run chunked2 2 --model chunked --steps 3 --warmup 2 --batch 128 --quality-steps 0 --recall 128
