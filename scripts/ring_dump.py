"""Reads an HRT_RING_DUMP file (renderer.cpp, written when the fold-ring watchdog fires) and summarises the
state of the sample queue's fold ring: tiles whose done mask has jobs the cursor has not reached (a fold
never run: lost hand-off) versus tiles missing completions, locks held, free-queue tail.

usage: python scripts/ring_dump.py dump.bin
"""
import sys

import numpy as np

raw = open(sys.argv[1], "rb").read()
ntiles, slots, nchunks, nctl = np.frombuffer(raw[:16], np.uint32)
cnt = np.frombuffer(raw[16:16 + 8 * 20], np.uint64)
ctl = np.frombuffer(raw[16 + 160:], np.uint32)
done = ctl[:2 * ntiles].view(np.uint64)
lock = ctl[2 * ntiles:4 * ntiles:2]
cursor = ctl[2 * ntiles + 1:4 * ntiles:2]
q = ctl[4 * ntiles:4 * ntiles + 4 * slots]
tail = ctl[4 * ntiles + 4 * slots]
full = (1 << int(nchunks)) - 1
print(f"tiles {ntiles} slots {slots} nchunks {nchunks}; queue {cnt[15]} jobs dealt; watchdog {cnt[16:19]}; "
      f"slots returned (tail) {tail}")
ncomplete = int(np.sum(cursor == nchunks))
print(f"tiles fully folded {ncomplete}; locks held {int(np.sum(lock != 0))}")
stuck = []
for t in range(ntiles):
    c = int(cursor[t])
    d = int(done[t])
    if c < nchunks and (d >> c) & 1:
        stuck.append((t, c, hex(d), int(lock[t])))
print(f"tiles whose next job is done but not folded: {len(stuck)}; first: {stuck[:10]}")
partial = [(t, int(cursor[t]), hex(int(done[t]))) for t in range(ntiles) if 0 < int(done[t]) and int(cursor[t]) < nchunks]
print(f"tiles with some jobs done, not all folded: {len(partial)}; first: {partial[:10]}")
