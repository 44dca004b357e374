#!/bin/bash
# Same-box A/B of two source trees on the driver-equivalent bench: the current tree and ./ab_old (a built
# checkout of an older commit, git-ignored), alternating:  bash scripts/ab_tree.sh [rounds=2]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for r in $(seq ${1:-2}); do
  for t in ab_old .; do
    (cd $t && timeout -k 10 400 python -u bench.py > /tmp/ab_tree.log 2> /tmp/ab_tree.err) || { echo "$t rc=$?"; tail -5 /tmp/ab_tree.err; exit 1; }
    echo "$t: $(tail -1 /tmp/ab_tree.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
  done
done
