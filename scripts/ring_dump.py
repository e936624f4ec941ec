"""Reads an HRT_RING_DUMP file (renderer.cpp, written when the fold-ring watchdog fires) and summarises the
state of the sample queue's fold ring: tiles whose next job is done but not folded (a lost hand-off) versus
tiles missing completions, locks held, the free-queue tail.

usage: python scripts/ring_dump.py dump.bin
"""
import sys

import numpy as np

raw = open(sys.argv[1], "rb").read()
ntiles, slots, nchunks, nctl = (int(v) for v in np.frombuffer(raw[:16], np.uint32))
cnt = np.frombuffer(raw[16:16 + 8 * 20], np.uint64)
ctl = np.frombuffer(raw[16 + 160:], np.uint32)
fold = ctl[:2 * ntiles].view(np.uint64)
tail = ctl[2 * ntiles + 4 * slots]
done = fold & np.uint64((1 << 48) - 1)
cursor = (fold >> np.uint64(48)) & np.uint64(0x7F)
lock = fold >> np.uint64(63)
print(f"tiles {ntiles} slots {slots} nchunks {nchunks}; queue {cnt[15]} jobs dealt; watchdog {cnt[16:20]}; "
      f"slots returned (tail) {tail}")
print(f"tiles fully folded {int(np.sum(cursor == nchunks))}; locks held {int(np.sum(lock != 0))}")
stuck = [(t, int(cursor[t]), hex(int(done[t]))) for t in range(ntiles)
         if int(cursor[t]) < nchunks and (int(done[t]) >> int(cursor[t])) & 1]
print(f"tiles whose next job is done but not folded: {len(stuck)}; first: {stuck[:10]}")
partial = [(t, int(cursor[t]), hex(int(done[t]))) for t in range(ntiles) if int(done[t]) and int(cursor[t]) < nchunks]
print(f"tiles with some jobs done, not all folded: {len(partial)}; first: {partial[:10]}")
