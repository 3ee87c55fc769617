#!/bin/bash
# The file path's host / device split (pipeline.plan_split) against host-only, end to end
# (tools/e2e_files.py): C2 batches of 5, 12 and 36 folders and a C5 (4K) batch of 12, three
# interleaved repetitions each, PLY bytes compared across runs.  Output: gpurun_out/<tag>/e2e_*.json
#   bash tools/e2e_split.sh <tag> [geom:views ...]     (default: c2:5 c2:12 c2:36 c5:12)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
shift
SPECS=("$@")
[ ${#SPECS[@]} -eq 0 ] && SPECS=(c2:5 c2:12 c2:36 c5:12)
mkdir -p "$O"
cd "$R"
for spec in "${SPECS[@]}"; do
  set -- ${spec/:/ }
  timeout -k 10 400 python tools/e2e_files.py --geom "$1" --views "$2" --runs auto:1,host:1 --reps 3 \
    --out "$O/e2e_$1_$2.json" > "$O/e2e_$1_$2.log" 2>&1 || { echo "[e2e_split] $spec FAILED"; tail -20 "$O/e2e_$1_$2.log"; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], {k: [r['s_per_view'] for r in v] for k, v in d['runs'].items()}, 'ply_equal', d['ply_bytes_equal_all_runs'], [r.get('split') for r in d['runs'].get('auto_group1', [])][:1])" "$O/e2e_$1_$2.json"
done
echo "[e2e_split] ALL_OK"
