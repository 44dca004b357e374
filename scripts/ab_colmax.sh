set -o pipefail
cd $GRAFT_REPO_ROOT
for cm in 84 28 42; do
  echo "== COLMAX $cm"
  MXR_HALO_COLMAX=$cm timeout -k 10 200 python -u scripts/bench_wgrad.py --only pyr || exit 1
  MXR_HALO_COLMAX=$cm timeout -k 10 200 python -u scripts/bench_halo.py --pipe "" --halo "" --hx32 "0,2,4,6" || exit 1
done
