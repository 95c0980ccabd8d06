# The queue-plumbed receiver (sdr_multi_run through bench.py --queue-child) at 1024 channels over the
# bench's device-generated input: L/R copies after the post stages (default) or on their own stream,
# at BLOCKS block counts, REPS interleaved rounds.  TAG=... [BLOCKS="25 60"] [REPS=2] bash tools/gpu/queue_ab.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-queue_ab}
mkdir -p $O
for rep in $(seq ${REPS:-2}); do
for nb in ${BLOCKS:-25 60}; do
for d2h in ${D2H:-post}; do
  SDR_MULTI_D2H=$d2h timeout -k 10 240 python bench.py --queue-child --channels ${CHANNELS:-1024} --blocks $nb \
      --cus ${CUS:-64} --cap-ch 0 --cap-out /tmp/q.npz > $O/q_${nb}_${d2h}_$rep.json 2> $O/q_${nb}_${d2h}_$rep.err; rc=$?
  echo "blocks $nb d2h $d2h: $(tail -1 $O/q_${nb}_${d2h}_$rep.json)"; [ $rc -eq 0 ] || { tail -5 $O/q_${nb}_${d2h}_$rep.err; exit $rc; }
done
done
done
