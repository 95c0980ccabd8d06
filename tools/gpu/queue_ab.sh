# The queue-plumbed receiver (sdr_multi_run through bench.py --queue-child) at 1024 channels over the
# bench's device-generated input, at BLOCKS block counts, REPS interleaved rounds: L/R copies after the
# post stages (D2H=post) or on their own stream (copy); output waits by event polling (SYNC=poll) or
# hipEventSynchronize (event).  TAG=... [BLOCKS="25 60"] [D2H=post] [SYNC=poll] [REPS=2] bash tools/gpu/queue_ab.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-queue_ab}
mkdir -p $O
for rep in $(seq ${REPS:-2}); do
  for nb in ${BLOCKS:-25 60}; do
    for d2h in ${D2H:-post}; do
      for sync in ${SYNC:-poll}; do
        f=$O/q_${nb}_${d2h}_${sync}_$rep
        SDR_MULTI_SYNC=$sync SDR_MULTI_D2H=$d2h timeout -k 10 240 python bench.py --queue-child --channels ${CHANNELS:-1024} \
            --blocks $nb --cus ${CUS:-64} --cap-ch 0 --cap-out /tmp/q.npz > $f.json 2> $f.err; rc=$?
        echo "blocks $nb d2h $d2h sync $sync: $(tail -1 $f.json)"; [ $rc -eq 0 ] || { tail -5 $f.err; exit $rc; }
      done
    done
  done
done
