#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 200 python scripts/diag_filter.py 2>&1 | grep -v amdgpu.ids
