#!/bin/bash
# Bench lines for the BASELINE configs other than the headline (1 GPU each).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
B="timeout -k 10 400 python bench.py --no-cpu-baseline --no-probe --steps 10 --warmup 3"
$B --layout vitb16 --total-clients 128 > gpurun_out/cfg4.log 2>&1 || { echo cfg4 failed; tail -5 gpurun_out/cfg4.log; exit 1; }
$B --layout gpt2s --total-clients 128 --in-dtype float16 --wave 32 > gpurun_out/cfg5.log 2>&1 || { echo cfg5 failed; tail -5 gpurun_out/cfg5.log; exit 1; }
$B --layout gpt2s --total-clients 128 --in-dtype float16 > gpurun_out/cfg5_onewave.log 2>&1 || { echo cfg5b failed; tail -5 gpurun_out/cfg5b.log; exit 1; }
$B --force-collective --chunks 4 > gpurun_out/cfg3_rank.log 2>&1 || { echo cfg3 failed; tail -5 gpurun_out/cfg3_rank.log; exit 1; }
$B --layout flat1m --total-clients 4 --steps 50 > gpurun_out/cfg1.log 2>&1 || { echo cfg1 failed; tail -5 gpurun_out/cfg1.log; exit 1; }
$B --total-clients 64 --in-dtype float64 --out-dtype float64 > gpurun_out/cfg2_f64.log 2>&1 || { echo f64 failed; exit 1; }
for f in cfg4 cfg5 cfg5_onewave cfg3_rank cfg1 cfg2_f64; do echo "$f: $(tail -1 gpurun_out/$f.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["achieved"], r["frac"], r["kernel_ms_per_step"], r["launches"])')"; done
