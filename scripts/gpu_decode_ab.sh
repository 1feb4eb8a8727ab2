#!/bin/bash
# hsz_decode2 variants (HIPSNAPSHOT_HSZ_DECODE2) A/B: rate of each, then two
# PMC passes (LDS counters, wait/issue counters) for the listed variants.
set -o pipefail
out=$PWD/gpurun_out/decode_ab
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD:$PYTHONPATH
for v in ${VARIANTS:-lds g00 g01 g40 g41}; do
  HIPSNAPSHOT_HSZ_DECODE2=$v timeout -k 10 120 python scripts/probes/hsz_decode_bench.py > $out/rate_$v.json 2> $out/rate_$v.err \
      || { echo RATE_FAIL $v; tail -20 $out/rate_$v.err; exit 1; }
  echo "$v $(cat $out/rate_$v.json)"
done
for v in ${PMC_VARIANTS:-lds g00}; do
  HIPSNAPSHOT_HSZ_DECODE2=$v TAG=_ab_${v}_lds bash scripts/gpu_decode_pmc.sh || exit 1
  HIPSNAPSHOT_HSZ_DECODE2=$v TAG=_ab_${v}_wait \
      COUNTERS="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU" \
      bash scripts/gpu_decode_pmc.sh || exit 1
done
