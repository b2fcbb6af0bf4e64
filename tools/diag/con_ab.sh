# same-box A/B of the product build (-ffp-contract=on) against -ffp-contract=fast (libf16env_fast.so,
# built by hand: f16_jsb_amd.build with OUT overridden and extra=('-ffp-contract=fast',))
set -e
O=gpurun_out
for i in 1 2 3; do
  for v in on fast; do
    L=f16_jsb_amd/libf16env.so; [ $v = fast ] && L=f16_jsb_amd/libf16env_fast.so
    timeout -k 10 200 env F16ENV_LIB=$L python bench.py --workload cfg5 --steps 1024 --warmup 20 --no-cpu-baseline > $O/ab5_${v}_$i.log 2>&1
    timeout -k 10 200 env F16ENV_LIB=$L python bench.py --steps 300 --warmup 20 --no-cpu-baseline --rollout-envs 0 > $O/ab3_${v}_$i.log 2>&1
  done
done
