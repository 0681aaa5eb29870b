/*
 * olpe_test.h -- test hooks of libolpe.so.  NOT part of the stable C-ABI (include/olpe.h):
 * the library exports them so that the repository's own tests can drive the failure and
 * hand-off paths on a real GPU; a consumer of the sampler has no use for them.
 */
#ifndef OLPE_TEST_H
#define OLPE_TEST_H

#include "olpe.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Failure paths of the collectives (olpe_comm.hip, olpe_comm_proto.h); persistent until
 * cleared with 0:
 *   1  the moments summary's preparation fails to allocate (OLPE_ENOMEM, before any
 *      collective: it travels in the uniformity check),
 *   2  the local summary launch fails after the check (both rounds still entered),
 *   3  the uniformity check's words fail to reach the device (the poisoned default is
 *      sent instead: every rank fails the check; applies to every collective),
 *   4  round 1's summed words fail to come back (the rank enters round 2 as failed). */
int olpe_moments_fault(olpe_ctx *ctx, int where);

/* Chunk hand-offs that provably wait (on != 0; 0 clears).  In every later launch that
 * cuts walkers into chunks (olpe_last_units > 1), a wave that finishes a walker's first
 * chunk holds its hand-off until some wave is waiting for a hand-off, and the launch runs
 * one workgroup more than the first chunks need, so that a later chunk starts while its
 * predecessor is held: olpe_unit_stats counts at least one wait whatever the dispatch
 * order.  The results are unchanged.  OLPE_EINVAL at launch when the workgroups would
 * not all be resident (too many walkers for the device). */
int olpe_test_hold_handoff(olpe_ctx *ctx, int on);

#ifdef __cplusplus
}
#endif
#endif /* OLPE_TEST_H */
