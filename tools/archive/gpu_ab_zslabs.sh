set -o pipefail
o=gpurun_out/r6c; mkdir -p $o
for w in 4 2; do for z in 0 3 6; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --emulate-world $w --zstats-slabs $z > $o/emu${w}_z$z.json 2> $o/emu${w}_z$z.err || { tail -5 $o/emu${w}_z$z.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$o/emu${w}_z$z.json').read().strip().splitlines()[-1]); print('emu$w z$z', d['ms_per_step'], {k: round(v, 2) for k, v in d['stage_ms'].items()})"
done; done
