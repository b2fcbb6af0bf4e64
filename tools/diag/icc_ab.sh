# same-box A/B of the reset-cache refill: libf16env_old.so (full refill pass) vs the product
# build (queued-lane refill); cfg5 bench, 1024 steps, interleaved
set -e
O=gpurun_out
for i in 1 2 3; do
  for v in new old; do
    L=f16_jsb_amd/libf16env.so; [ $v = old ] && L=f16_jsb_amd/libf16env_old.so
    timeout -k 10 200 env F16ENV_LIB=$L python bench.py --workload cfg5 --steps 1024 --warmup 20 --no-cpu-baseline > $O/iccab_${v}_$i.log 2>&1
  done
done
