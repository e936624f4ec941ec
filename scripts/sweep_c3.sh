set -e
for sb in 16 20 28; do LIBS=lib/libhrt.so scripts/exp_cfg.sh c3 "--suspend-below $sb" | sed "s/^/sb$sb /"; done
LIBS=lib/libhrt.so scripts/exp_cfg.sh c3 "" | sed "s/^/sb24 /"
LIBS=lib/libhrt.so scripts/exp_cfg.sh c3 "--job-frames 64" | sed "s/^/jf64 /"
