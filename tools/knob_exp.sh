#!/bin/bash
# A/B of launch knobs on the 9-mer pass: one bench run (3 timed steps) per setting, in the
# same GPU call.  usage: tools/knob_exp.sh OUTDIR "VAR=a VAR2=b" "VAR=c" ...
out=$1; shift
mkdir -p "$out"
i=0
for setting in "$@"; do
  i=$((i+1))
  env $setting timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-full-cv --no-cpu-baseline \
      > "$out/knob$i.json" 2> "$out/knob$i.err" || { echo "setting [$setting] failed"; tail -3 "$out/knob$i.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$out/knob$i.json')); r=d['roofline']; print('[$setting]', round(d['ms_per_step'],2), 'ms/step', round(r['kernel_ms_per_pass'],2), 'kernel ms')"
done
