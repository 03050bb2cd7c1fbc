#!/bin/bash
# Zeroscope evidence (per-shape table of one 576x320x24 clip, one PMC pass) and the VAE-graph
# stream-serialisation measurement (scripts/graph_serialisation.py, eager VAE vs graph-replayed).
set -o pipefail
TAG=${1:-vidg}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "== stag2 prefetch A/B $(date +%T)"
timeout -k 10 400 python -u scripts/stag2_pd_ab.py --rounds 5 > $O/stag2_pd_ab.jsonl 2>$O/stag2_pd_ab.err || { tail -20 $O/stag2_pd_ab.err; exit 1; }
cut -c1-200 $O/stag2_pd_ab.jsonl
for v in eager graph; do
  echo "== vae $v $(date +%T)"
  a=""; [ $v = graph ] && a="--vae-graph"
  timeout -k 10 400 python -u scripts/graph_serialisation.py $a --groups 3 --json $O/graph_ser_$v.json > $O/graph_ser_$v.log 2>&1 \
    || { tail -20 $O/graph_ser_$v.log; exit 1; }
  head -3 $O/graph_ser_$v.log | cut -c1-300
done
for v in 0 1; do
  echo "== k2 prior graph $v $(date +%T)"
  ARB_PRIOR_GRAPH=$v timeout -k 10 400 python bench.py --model kandinsky2 --steps 4 --warmup 1 > $O/k2_pg$v.log 2>$O/k2_pg$v.err \
    || { tail -20 $O/k2_pg$v.err; exit 1; }
  tail -1 $O/k2_pg$v.log | cut -c1-160
done
for c in 3 4; do
  echo "== zeroscope c$c $(date +%T)"
  timeout -k 10 500 python bench.py --model zeroscopev2xl --steps 3 --warmup 1 --concurrent $c > $O/zs_c$c.log 2>$O/zs_c$c.err \
    || { tail -20 $O/zs_c$c.err; exit 1; }
  tail -1 $O/zs_c$c.log | cut -c1-160
done
echo "== layer_prof zeroscope $(date +%T)"
timeout -k 10 400 python scripts/layer_prof.py --model zeroscopev2xl --steps 2 --md $O/shapes_zeroscope.md \
  --json $O/shapes_zeroscope.jsonl > $O/lp_zs.log 2>&1 || { tail -30 $O/lp_zs.log; exit 1; }
head -1 $O/shapes_zeroscope.md | cut -c1-300
echo "== pmc zeroscope $(date +%T)"
MODEL=zeroscopev2xl STEPS=3 bash scripts/gpu_pmc_bench.sh ${TAG}_pmc_zs
echo "== done $(date +%T)"
