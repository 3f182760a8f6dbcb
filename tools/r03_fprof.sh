# Phase profile of the one-launch small decode (C2 and neighbours): bash tools/r03_fprof.sh TAG
O=gpurun_out/r03_$1; mkdir -p $O
for g in "1 16 4" "1 16 8" "4 16 4" "1 64 8"; do
  timeout -k 10 60 tools/tc_profile fused $g >> $O/fused_phases.log 2>&1 || exit $?
done
cat $O/fused_phases.log
