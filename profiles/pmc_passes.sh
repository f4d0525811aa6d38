#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 process per pass, counters only
# with kernel dispatch records; no API/system tracing in the same pass).
# usage: bash profiles/pmc_passes.sh <outdir> <pass-name>=<c1,c2,...> ...
set -e
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/$1; shift
mkdir -p "$OUT"
for spec in "$@"; do
  name=${spec%%=*}; ctrs=${spec#*=}
  timeout -k 10 240 rocprofv3 --pmc ${ctrs//,/ } --kernel-include-regex "k_walker_rev|k_walker|k_moved" \
    -d "$OUT/$name" -o "$name" -f csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-ecp --no-adam --no-dmc \
    > "$OUT/$name.log" 2>&1
  echo "pass $name done"
done
