/*
 * hrt_testing.h — test-only entry points of libhrt.so (fault injection). Not part of the drop-in surface
 * (include/hrt.h): the reference has nothing to bind here, and a product caller never needs
 * them. The parity suite uses them to drive the sample queue's rare paths on a healthy device.
 */
#ifndef HRT_TESTING_H
#define HRT_TESTING_H

#include "hrt.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ring_slots_max: the fold ring gets at most this many job slots (rounded down to a power of two; 0 = no cap),
 *   so that nearly every job waits for one.
 * fail_alloc_above_mb: colour-fold allocations above this many MiB fail as a refused hipMalloc would (0 = off);
 *   the draw then shrinks them.
 * Both stay set until changed; a new renderer starts with both 0. */
int rt_testing_set_faults(rt_renderer *r, uint32_t ring_slots_max, uint32_t fail_alloc_above_mb);

#ifdef __cplusplus
}
#endif
#endif /* HRT_TESTING_H */
