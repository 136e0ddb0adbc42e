set -e
mkdir -p gpurun_out
o=gpurun_out/ba_shares.txt; : > $o
for sh in "4,1" "6,1" "8,1" "6,2" "8,2" "4,2"; do
  echo "== shares $sh" >> $o
  DPVO_BA_SHARES=$sh timeout -k 10 120 python scripts/ba_window_phases.py cfg2 2 2>/dev/null | grep -v "^/opt" >> $o
done
