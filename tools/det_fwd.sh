# run-to-run determinism of forward variants (build/fwd_*): 100 launches each, hashes vs the first
set -e
for v in "$@"; do echo "== $v"; timeout -k 5 120 build/fwd_$v 20 100; done
