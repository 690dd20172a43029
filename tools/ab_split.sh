#!/bin/bash
# A/B the pair_ring role split per pair kind (tools/ab_option.py; kernel classes 12 mid, 13 top, 14 bot)
out=${1:-gpurun_out/ab_split}
mkdir -p $out
timeout -k 10 200 python -u tools/ab_option.py pair_split_mid 16,17,18,19,20 --rounds 2 --steps 100 --kclass 12 > $out/mid.txt 2>&1 &&
timeout -k 10 200 python -u tools/ab_option.py pair_split_top 16,17,18,19 --rounds 2 --steps 100 --kclass 13 > $out/top.txt 2>&1 &&
timeout -k 10 200 python -u tools/ab_option.py pair_split_bot 16,17,18,19,20 --rounds 2 --steps 100 --kclass 14 > $out/bot.txt 2>&1
