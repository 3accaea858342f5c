#!/bin/bash
# Rehearsal of the N>1 bench path on one GPU: 2 and 4 ranks share the card,
# host (gloo) collectives; the gathered image is checked bit-exact vs a 1-GPU frame
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${TAG:-gloo}; mkdir -p $OUT
for n in 2 4; do
  RTMI_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 3 --warmup 1 --no-cpu-baseline --no-exec-counts > $OUT/gloo$n.json 2> $OUT/gloo$n.err || { tail -5 $OUT/gloo$n.err; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$OUT/gloo$n.json') if l.startswith('{')][-1]); print($n, d['value'], d['ms_per_step'], d.get('gather_check'), json.dumps(d.get('dist')))"
done
