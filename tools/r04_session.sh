# Round-4 final evidence (r04z): rocprof stats + PMC passes + bench line +
# smoke (tools/profile_round.sh), then the e2e kernel trace of run_epoch
# summarised per training batch (the raw trace stays on the box).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/profile_round.sh r04z
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/r04z_e2etrace -o run -- python3 tools/e2e_profile.py --no-cprofile > gpurun_out/r04z_e2etrace.log 2>&1
python3 tools/trace_batch.py "$(find /tmp/r04z_e2etrace -name '*kernel_trace.csv' | head -1)" > gpurun_out/r04z_e2e_train_batch_kernels.txt 2>&1
