# The queue-plumbed receiver (sdr_multi_run through bench.py --queue-child) at 1024 channels over the
# bench's device-generated input, at BLOCKS block counts, REPS interleaved rounds: L/R copies after the
# post stages (D2H=post) or on their own stream (copy); both consumers' post stages on one stream
# (POSTS=1) or one each (2).  TAG=... [BLOCKS="25 60"] [D2H=post] [POSTS=1] [REPS=2] bash tools/gpu/queue_ab.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-queue_ab}
mkdir -p $O
for rep in $(seq ${REPS:-2}); do
  for nb in ${BLOCKS:-25 60}; do
    for d2h in ${D2H:-post}; do
      for posts in ${POSTS:-1}; do
        f=$O/q_${nb}_${d2h}_p${posts}_$rep
        SDR_MULTI_POSTS=$posts SDR_MULTI_D2H=$d2h timeout -k 10 240 python bench.py --queue-child --channels ${CHANNELS:-1024} \
            --blocks $nb --cus ${CUS:-64} --cap-ch 0 --cap-out /tmp/q.npz > $f.json 2> $f.err; rc=$?
        echo "blocks $nb d2h $d2h posts $posts: $(python3 -c "import json,sys; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); d.pop('pll_block_us'); d.pop('iq_sha'); print(json.dumps(d))")"; [ $rc -eq 0 ] || { tail -5 $f.err; exit $rc; }
      done
    done
  done
done
