#!/bin/bash
# GPU box: A/B of bench.py variants.  VARIANTS: ';'-separated "ENV=.. ARGS" items,
# e.g. VARIANTS='|--overlap|--overlap --comm split'.  Each run under its own limit.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab}
mkdir -p $O
IFS='|' read -ra VS <<< "$VARIANTS"
i=0
for v in "${VS[@]}"; do
  i=$((i+1))
  envs=$(echo "$v" | tr ' ' '\n' | grep '=' | tr '\n' ' ')
  args=$(echo "$v" | tr ' ' '\n' | grep -v '=' | tr '\n' ' ')
  env $envs timeout -k 10 300 python3 -u bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline --no-secondary $args > $O/v$i.log 2>&1 || { echo "variant $i [$v] failed"; tail -5 $O/v$i.log; exit 1; }
  echo "[$v] $(tail -1 $O/v$i.log | grep -o '"ms_per_step": [0-9.]*')"
done
