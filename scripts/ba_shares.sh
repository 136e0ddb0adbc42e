set -e
mkdir -p gpurun_out
o=gpurun_out/ba_shares.txt; : > $o
for sh in "1,1" "2,1" "3,1" "4,1"; do
  echo "== shares $sh" >> $o
  DPVO_BA_SHARES=$sh timeout -k 10 120 python scripts/ba_window_phases.py cfg2 2 2>/dev/null | grep -v "^/opt" >> $o
done
