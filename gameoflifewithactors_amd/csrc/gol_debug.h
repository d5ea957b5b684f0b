/*
 * gol_debug.h -- test and A/B knobs of libgol_hip.so (internal: not part of the drop-in boundary include/gol/gol.h).
 *
 * These change how a pass is launched or let a test drive a rare state early; unlike gol.h's gol_set_option names,
 * some of them are not results-neutral by themselves (a spin limit of one poll makes a hand-off time out and the
 * board invalid), so the F# drop-in does not bind them.  The tests and the A/B tools reach them through ctypes.
 *   "coop_epoch" 0..65535       the tag epoch of the last persistent launch (the next runs at value + 1); setting it
 *                               clears the hand-off granules, so no stale granule can match a later launch's tag
 *   "coop_spin_limit" 0 | n     polls before a hand-off wait gives up and marks the board invalid (0: ~2 s)
 *   "coop_r" 1..8               cooperative pass: rows per wave at least (A/B)
 *   "resident_threads" 1024 | 256  LDS-resident pass workgroup size (A/B)
 *   "coop_launch" 0 | 1         persistent passes by hipLaunchKernel after a residency check (0), or by
 *                               hipLaunchCooperativeKernel (1; DESIGN.md 6 "Exit under rocprofv3")
 *   "lanes_launches"            (read-only) launches of the rows-on-lanes pass on this board
 * Unknown names return GOL_ERR_INVALID.
 */
#ifndef GOL_DEBUG_H
#define GOL_DEBUG_H

#include <stdint.h>

#include "gol/gol.h"

#ifdef __cplusplus
extern "C" {
#endif

int gol_debug_set_option(gol_board* b, const char* name, int64_t value);
int gol_debug_get_option(gol_board* b, const char* name, int64_t* value);
/* The names above, comma-separated (the library's own list: _lib.DEBUG_OPTIONS is tested against it). */
const char* gol_debug_option_names(void);
/* Level-pipelined pass (gol_pipe.hip): its plan for a strip pass with `wgs` resident workgroups (0: the device's) and
 * the violations a host walk of it finds -- plan[15] = nstrips, rem, rq, rp, ngroups, grows, pk_lo, pk_hi, npk, nrem,
 * P, split1, split2, grid, violations -- and the library's own error word of its strip passes (read and cleared). */
int gol_debug_pipe_plan(const gol_strip* s, int k, int64_t out_begin, int64_t out_end, int64_t wgs, int64_t* plan,
                        int64_t n);
int gol_debug_pipe_errors(int* out);

#ifdef __cplusplus
}
#endif
#endif /* GOL_DEBUG_H */
