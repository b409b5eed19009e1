# two-rank gloo rehearsal of bench.py's run_epoch line, full stderr kept
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --e2e-only --dist-backend gloo \
  > gpurun_out/r06c_e2e2.out 2> gpurun_out/r06c_e2e2.err
echo "rc=$?" >> gpurun_out/r06c_e2e2.out
