# (1) trainer-only ms per SGD step under fp16 autocast (the reference's) and bf16 autocast, graphed and
# eager; (2) config 3 in steady state (scripts/gpu_config3_steady.sh: one game generation of warm-up,
# 6 timed plies, 4 no-dedup twin plies).
# (--trainer-dtype-ab and the bf16 trainer option belong to commit 329bc68's tree; bf16 was measured
# slower, profiles/r04/trainer/autocast_dtype_ab.json, and removed.)
set -u
O=gpurun_out/r04i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 scripts/bench_train.py --trainer-dtype-ab > $O/train_dtype.json 2> $O/train_dtype.err || { tail -5 $O/train_dtype.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/train_dtype.json'))
for r in d['trainer_only']: print('trainer graph', r['train_graph'], 'autocast', r['train_autocast'], round(r['ms_per_sgd_step'],2), 'ms', round(r['last_loss'],4))"
TAG=r04 bash scripts/gpu_config3_steady.sh
