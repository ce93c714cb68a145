#!/bin/bash
# Interleaved A/B of runtime variants selected by environment settings (GPU box).
# usage: tools/ab_env.sh "<bench args>" "ENV=a" "ENV=b" ...
args=$1; shift
for rep in 1 2 3; do
  for v in "$@"; do
    env $v timeout -k 10 120 python bench.py --cpu-baseline 0 $args 2>/dev/null | \
      python3 -c "import sys,json; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$v', 'rep $rep', round(d['value']), 'chk', d['var_checksum'], ' '.join(f'{n}_us {v[\"avg_us\"]:.1f}' for n,v in k.items()))"
  done
done
