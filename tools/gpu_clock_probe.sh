#!/bin/bash
# GPU box: sample the GPU clocks / power (rocm-smi, 1 Hz) while the isolated attention probe and
# then one bench iteration run, to compare the effective clock of the two.
out=gpurun_out/${1:-clk}; mkdir -p $out
( while true; do date +%s.%N; rocm-smi --showclocks --showpower 2>/dev/null | grep -E "sclk|fclk|mclk|Power"; sleep 1; done ) > $out/smi.txt 2>&1 &
sampler=$!
echo "probe_start $(date +%s.%N)" > $out/marks.txt
PRFL_PROF_WARM_S=10 PRFL_PROF_L=73920 timeout -k 10 150 python3 tools/attn_layout_probe.py 5 > $out/probe.txt 2>&1
rc=$?
echo "probe_end $(date +%s.%N)" >> $out/marks.txt
if [ $rc = 0 ]; then
  timeout -k 10 600 python -u bench.py --no-cpu-baseline --warmup 0 --steps 1 > $out/bench.json 2> $out/bench.err
  rc=$?
fi
echo "bench_end $(date +%s.%N)" >> $out/marks.txt
kill $sampler
grep "L=" $out/probe.txt; cat $out/marks.txt
exit $rc
