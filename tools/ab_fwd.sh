# A/B of forward variants in the standalone harness (build/fwd_<name>): bash tools/ab_fwd.sh name...
set -e
for i in 1 2; do
for v in "$@"; do echo "== $v"; timeout -k 5 60 build/fwd_$v 200; done
done
