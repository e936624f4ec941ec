#!/usr/bin/env bash
# job_frames sweep for the triangle/mixed programs (C4, C5 at 256 frames) and C3.
set -e
for jf in 32 64; do LIBS=lib/libhrt.so scripts/exp_cfg.sh c4 "--job-frames $jf" | sed "s/^/jf$jf /"; done
LIBS=lib/libhrt.so scripts/exp_cfg.sh c5 "--frames 256 --job-frames 64" | sed "s/^/jf64 /"
for jf in 16 32; do LIBS=lib/libhrt.so scripts/exp_cfg.sh c3 "--job-frames $jf" | sed "s/^/jf$jf /"; done
