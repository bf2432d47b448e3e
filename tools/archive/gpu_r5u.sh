#!/bin/bash
# round 5 late: the round-end style run (every GPU test, smoke, the full bench line with config
# lines, kernel traces) + the emulated world-8 / 4 / 2 rank steps
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu_roundend.sh r5u || exit 1
o=gpurun_out/r5u
python3 -c "import json; d=json.load(open('$o/bench.json')); [print(k, json.dumps(d[k])[:400]) for k in ('config_b','config_d','config_e')]"
for w in 8 4 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --emulate-world $w > $o/emu$w.json 2> $o/emu$w.err || { tail -5 $o/emu$w.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$o/emu$w.json').read().strip().splitlines()[-1])
print('emu$w', d['ms_per_step'], {k: round(v,2) for k,v in d.get('stage_ms',{}).items()})"
done
