# A/B of the forward's epilogue forms in the standalone harness (build/fwd_{base,magic}[clk])
set -e
for i in 1 2; do
for v in base magic; do echo "== $v"; timeout -k 5 60 build/fwd_$v 200; done
done
for v in baseclk magicclk; do echo "== $v"; timeout -k 5 60 build/fwd_$v 2000; done
