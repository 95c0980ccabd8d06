# The queue-plumbed receiver (sdr_multi_run through bench.py --queue-child) at 1024 channels over the
# bench's device-generated input, at BLOCKS block counts, REPS interleaved rounds, once per setting in
# ENVS (space-separated NAME=value[,NAME=value] items; "-" = none), e.g. the engine's A/B knobs
# SDR_MULTI_EDGES (0: no all-CU fill/drain stream), SDR_MULTI_POSTS (2: a post stream per consumer),
# SDR_MULTI_D2H (copy: L/R copies on their own stream), SDR_MULTI_SYNC (event: hipEventSynchronize).
#   TAG=... [BLOCKS="25 60"] [ENVS="- SDR_MULTI_EDGES=0"] [REPS=2] bash tools/gpu/queue_ab.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-queue_ab}
mkdir -p $O
for rep in $(seq ${REPS:-2}); do
  for nb in ${BLOCKS:-25 60}; do
    i=0
    for ev in ${ENVS:--}; do
      i=$((i+1))
      f=$O/q_${nb}_e${i}_$rep
      envs=""; [ "$ev" != "-" ] && envs=$(echo "$ev" | tr ',' ' ')
      env $envs timeout -k 10 240 python bench.py --queue-child --channels ${CHANNELS:-1024} \
          --blocks $nb --cus ${CUS:-64} --cap-ch 0 --cap-out /tmp/q.npz > $f.json 2> $f.err; rc=$?
      [ $rc -eq 0 ] || { tail -5 $f.err; exit $rc; }
      echo "blocks $nb [$ev]: $(python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); d.pop('pll_block_us'); d.pop('iq_sha'); print(json.dumps(d))")"
    done
  done
done
