set -e
for cfg in ${CFGS:-"3 384" "4 384" "6 384" "4 512" "8 512"}; do
  set -- $cfg
  timeout -k 10 200 python bench.py --no-cpu-baseline --lba-steps 0 --pose-frames 0 --tri-pairs 0 --aux 0 --p1080-frames 0 --latency-frames 0 --iso-reps 0 --stage-timing 0 --parity-check 0 --streams $1 --frames $2 > gpurun_out/st_$1_$2.json 2>/dev/null
  python3 -c "import json;d=json.loads(open('gpurun_out/st_$1_$2.json').read().strip().splitlines()[-1]);print('$1 streams $2 frames', d['value'], d['ms_per_step'])"
done
