# config A/B across worktrees of earlier commits (.wt_<commit>/, each with its own built libjmhip.so):
#   bash tools/ab_trees.sh TAG CONFIG commit...     (runs each tree's own bench.py, then this tree's)
TAG=$1; CFG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
for c in "$@" head; do
  if [ $c = head ]; then d="$R"; else d="$R/.wt_$c"; fi
  (cd "$d" && timeout -k 10 240 python bench.py --config $CFG --steps 60 --no-cpu-baseline --no-host-path > "$R/gpurun_out/${TAG}_$c.json" 2> "$R/gpurun_out/${TAG}_$c.err")
  echo "$c rc=$? $(grep -o '"value": [0-9.]*' "$R/gpurun_out/${TAG}_$c.json" | head -1)"
done
