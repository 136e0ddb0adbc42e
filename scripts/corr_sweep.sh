set -e
mkdir -p gpurun_out
o=gpurun_out/corr_diag.txt; : > $o
for b in corr_bench corr_bench_NO_MMA corr_bench_NO_LOAD; do
for args in "1 3 1 512" "1 0 1 512" "1 0 4 2048"; do
  echo "== $b $args" >> $o
  timeout -k 5 60 ./scripts/micro/$b $args 1 2>&1 | head -5 >> $o
done
done
