# rehearse the N>1 bench path on the one-GPU box: 2 ranks on cuda:0, gloo gather, image check
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --steps 1 --warmup 1 --spp 32 --backend gloo --check-image > gpurun_out/mr_gloo2.log 2>&1
rc=$?; grep -h "check_image\|\"value\"" gpurun_out/mr_gloo2.log | cut -c1-400; exit $rc
