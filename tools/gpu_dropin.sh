# drop-in latency at notebook sizes (tools/bench_dropin.py)
set -o pipefail
mkdir -p gpurun_out/dropin
timeout -k 10 400 python -u tools/bench_dropin.py ${DROPIN_ARGS:-} > gpurun_out/dropin/dropin.json 2> gpurun_out/dropin/dropin.err || { tail -20 gpurun_out/dropin/dropin.err; exit 1; }
grep -v amdgpu.ids gpurun_out/dropin/dropin.err
