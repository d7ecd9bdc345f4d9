#!/bin/bash
# rocprofv3 FETCH_SIZE / WRITE_SIZE passes (one counter per run, MI355X_MICROARCH.md HBM recipe) of the
# F=hid SpMM on one rank's share of the partitioned bench workloads (c2 weak scaling and c4, N = 2, 4, 8),
# plus the whole c4 graph at N = 1 -- the sources of bench.py's roofline.traffic at every N.
# Summaries: gpurun_out/pmc_rs/r04_pmc_rs_*.json (copy into profiles/).  Stops at the first failing pass.
set -u
OUT=gpurun_out/pmc_rs
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {  # pass <name> <counter> -- <program...>
  local name=$1 counter=$2; shift 3
  timeout -s KILL 240 rocprofv3 --pmc $counter --output-format csv -d "$OUT/$name" -o run -- "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit 3
}
for fam in ${FAMILIES:-c2 c4}; do
  for n in ${WORLDS:-2 4 8}; do
    pass ${fam}_n${n}_fetch FETCH_SIZE -- python3 tools/pmc_rank_share.py --family $fam --world $n
    pass ${fam}_n${n}_write WRITE_SIZE -- python3 tools/pmc_rank_share.py --family $fam --world $n
    python3 tools/pmc_summary.py "$OUT/${fam}_n${n}_fetch" "$OUT/${fam}_n${n}_write" "$OUT/r04_pmc_rs_${fam}_n${n}.json" \
      "$(python3 tools/pmc_rank_share.py --family $fam --world $n --print-key)" | tail -1
  done
done
if [ -z "${SKIP_C4_N1:-}" ]; then
  pass c4_n1_fetch FETCH_SIZE -- python3 bench.py --config c4 --steps 2 --warmup 1 --profile-only
  pass c4_n1_write WRITE_SIZE -- python3 bench.py --config c4 --steps 2 --warmup 1 --profile-only
  python3 tools/pmc_summary.py "$OUT/c4_n1_fetch" "$OUT/c4_n1_write" "$OUT/r04_pmc_spmm_c4_n1.json" \
    "$(python3 bench.py --config c4 --print-workload)" | tail -1
fi
echo pmc_rank_shares done
