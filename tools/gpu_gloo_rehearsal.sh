#!/bin/bash
# Rehearsal of the N>1 bench path on one GPU: bench.py
# --gpus N through its OWN launcher (launch(): a torch.distributed.run child
# of a parent that never touches the GPU), RTMI_DIST_BACKEND=gloo so the N
# ranks share the card and the collectives run on host copies.  N = 2, 3
# (800 rows ragged over 3 ranks) and 8; every line carries dist (backend,
# world size, per-rank kernel / gather / segments / wall) and gather_check
# (the gathered image against rank 0's own whole frame, bit for bit).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-gloo}; mkdir -p $OUT
for n in ${RANKS:-2 3 8}; do
  RTMI_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus $n --steps 3 --warmup 1 --no-cpu-baseline --no-exec-counts > $OUT/gloo$n.json 2> $OUT/gloo$n.err || { tail -5 $OUT/gloo$n.err; exit 1; }
  python -c "import json; ls=open('$OUT/gloo$n.json').read().splitlines(); assert len(ls) == 1, 'stdout is not one line'; d=json.loads(ls[0]); print($n, d['n_gpus'], d['value'], d['ms_per_step'], 'one_shot', d.get('one_shot_msamples_per_s'), d.get('gather_check'), json.dumps(d.get('dist')))"
done
