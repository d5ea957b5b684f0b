// gol_internal.h -- launcher prototypes shared by the kernel files and gol_capi.cpp (not installed).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gol {

// Geometry of one streaming pass over a bit-packed buffer (gol_step.hip).
struct StreamArgs {
    int64_t words;      // board words per row (board width / 32)
    int64_t pitch;      // words per buffer row (multiple of ilv)
    int64_t rows;       // owned rows (in wrap mode: all rows of the buffer)
    int64_t ghost;      // halo rows stored above and below the owned rows (0 in wrap mode)
    int64_t y0;         // global row index of owned row 0 (bounded masking, strips)
    int64_t height;     // global board height
    int64_t out_begin;  // owned rows [out_begin, out_end) are produced
    int64_t out_end;
    int64_t seg;        // rows per wave segment (plan_stream)
    int64_t nstrips;    // filled by plan_stream
    int64_t nsegs;      // filled by plan_stream
    int32_t ilv;        // words per interleaved block (gol_layout.h): 1, 2 or 4
    int32_t split;      // filled by plan_stream: pair split (older wave's share of a pair segment, 1/65536;
                        // 0 = one segment per wave)
    int32_t spare;      // waves to leave free for concurrent launches (plan_stream)
    int32_t split_opt;  // 0: the engine's pair split; > 0: this split (1/65536); < 0: none (board option "split")
    int32_t split2;     // filled by plan_stream: three-wave groups, the middle wave's share of the middle + youngest
                        // waves' rows (1/65536); 0 = the same ratio as the pair split (geometric shares)
    int32_t split2_opt; // 0: the engine's; > 0: this value (board option "split2")
    int64_t seg_opt;    // 0: plan the segment length; > 0: rows per segment (board option "seg_rows")
    // Seam geometry (torus, filled by plan_stream; gol_step.hip): `nstrips` strips of 63 stored blocks plus one seam
    // lane holding both halos, and the rem = nblocks - 63 * nstrips blocks left over in remainder waves that pack
    // rem_p sub-strips of (rem + 2) lanes, each on its own row segment.
    int32_t seam;       // 1: seam geometry; 0: strips of 62 stored blocks with a halo lane on each side
    int32_t rem;        // remainder blocks per row (0..62)
    int32_t rem_p;      // remainder sub-strips per wave
    int64_t rem_units;  // remainder units (after the nstrips * nsegs main units)
    int64_t rem_mid;    // segments 1 .. rem_mid share remainder waves (the others have one each)
    int32_t seam_opt;   // board option "seam": 0 = the engine's choice, < 0 = off
    int32_t rag_bits;   // ragged rows (width not a multiple of 32): cells in a row's last word (1..31); 0 otherwise
    int32_t rag_origin; // filled by plan_stream: ragged torus strips start at ring position -rag_origin
    int64_t rag_w;      // bounded ragged rows: the board's width in cells (cells past it are dead); 0 otherwise
    // Level-pipelined pass (gol_pipe.hip: torus, ilv 4, K = 16 / 32): the board options "pipe_split" / "pipe_split2"
    // (0 = the engine's, > 0 this share (1/65536), < 0 equal shares), and where a timed-out ring wait is reported (a
    // board's error word; null: the library's own, gol_debug_pipe_errors)
    int32_t pipe_split_opt;
    int32_t pipe_split2_opt;
    int* pipe_err;
};

// Geometry of one level-pipelined pass (gol_pipe.hip), filled from StreamArgs and plan_pipe.
struct PipeArgs {
    int64_t words, pitch, rows, ghost, out_begin, out_end;  // as StreamArgs
    int64_t nblocks;   // blocks of 4 words per row
    int64_t nstrips;   // full strips of 62 stored blocks (bounded: the first and last of them store 63, at the edges)
    int32_t rem;       // blocks past the full strips (bounded: before the last one) in remainder workgroups, 0..30
    int32_t rq;        // lanes per remainder sub-strip (rem + 2)
    int32_t rp;        // remainder sub-strips per wave
    int32_t P;         // pipelines per workgroup
    int64_t ngroups;   // row groups per strip (a workgroup each), of grows rows (the last may be shorter)
    int64_t grows;
    int64_t pk_lo, pk_hi;  // groups [pk_lo, pk_hi) share remainder workgroups rp at a time; the others have one each
    int64_t npk;       // packed remainder workgroups
    int64_t nrem;      // remainder workgroups in all (after nstrips x ngroups)
    int32_t split1;    // the oldest pipeline's share of a pair (1/65536, 0 = equal shares)
    int32_t split2;    // after the second-oldest (0 = split1)
    int64_t spare_waves;  // waves to leave free for concurrent launches
    int64_t spin_limit;   // polls before a ring wait gives up (0 = the default)
    int* err;             // set non-zero by a wait that gave up
    int64_t wgs_opt;      // planning without a device (tests): resident workgroups (0 = the device's)
    // Bounded boards (Script.fsx:6-13): strips laid out with the board's edges on a wave's outer lanes (zero-filled
    // lane moves), and the rows [live_lo, live_hi) (owned-row coordinates) the only live ones: rows outside stay dead
    int32_t bounded;
    int32_t live_lo, live_hi;
};

// ---- gol_step.hip
bool stream_supported(int k, int ilv);
int stream_max_k(int ilv);
// the deepest supported depth <= cap and <= n for rows of `words` words (words 0: never a level-pipelined depth)
int stream_largest_k(int64_t n, int cap, int ilv, int64_t words = 0, bool bounded = false);
// rag_bits: cells in the last word of a ragged row (words = ceil(W / 32), ilv 1), 0 for whole-word rows
int64_t stream_strips(int64_t words, int ilv, int k, bool bounded, int rag_bits = 0);
int stream_pair_split(int k, int ilv, bool bounded, bool wrap, bool single);
int stream_split2(int k, int ilv, bool bounded, bool wrap, bool single);
int stream_wpb(int64_t words, int k, int ilv, bool bounded, bool wrap, int rag_bits = 0);
// fills nstrips / nsegs / seg (one balanced round of resident waves unless a.seg_opt -- the "seg_rows" option -- is set)
void plan_stream(StreamArgs& a, int k, bool bounded, bool wrap);
hipError_t launch_stream_step(const uint32_t* src, uint32_t* dst, StreamArgs a, int k, bool bounded, bool wrap,
                              hipStream_t s);
// PipeArgs of a pass over StreamArgs' buffer (split options, error word, spare waves, the live rows of a bounded board)
PipeArgs pipe_args(const StreamArgs& a, bool bounded);

// ---- gol_pipe.hip: the level-pipelined deep pass (ilv 4, K = 16 or 32; torus and bounded rows of >= 62 / 64 blocks;
// a.bounded selects the bounded geometry in the functions below)
bool pipe_supported(int k);
bool pipe_applies(int64_t words, int ilv, int k, bool bounded, int rag_bits);
int pipe_default_split(int k);
void plan_pipe(PipeArgs& a, int k, bool wrap, int64_t spare_waves);
int64_t pipe_grid(const PipeArgs& a);  // workgroups of a planned pass (16 waves each)
hipError_t launch_pipe_step(const uint32_t* src, uint32_t* dst, PipeArgs a, int k, bool wrap, hipStream_t s);
int* pipe_error_word();  // the library's own error word (strip passes), device memory
// Walks a planned pass on the host (tests): every output (row, block) stored, every row a packed remainder sub-strip
// reads inside the buffer without a wrap or clamp, lane offsets in 32 bits.  Returns the violations found.
int64_t pipe_check_plan(const PipeArgs& a, int k, bool wrap);

// ---- gol_formats.hip
hipError_t launch_bytes_step(const uint8_t* src, uint8_t* dst, int64_t W, int64_t H, bool bounded, hipStream_t s);
hipError_t launch_pack(const uint8_t* cells, uint32_t* words, int64_t W, int64_t rows, int64_t pitch, int64_t row0,
                       int ilv, hipStream_t s);
// byte board (any width W) <-> consecutive words, `pitch` words per row: bit b of word j = cell 32 j + b, cells past
// W (and whole words past ceil(W / 32)) zero; unpack writes 0 / 1 for the W cells of each row
hipError_t launch_pack_ragged(const uint8_t* cells, uint32_t* words, int64_t W, int64_t H, int64_t pitch, hipStream_t s);
hipError_t launch_unpack_ragged(const uint32_t* words, uint8_t* cells, int64_t W, int64_t H, int64_t pitch,
                                hipStream_t s);
hipError_t launch_unpack(const uint32_t* words, uint8_t* out, int64_t W, int64_t rows, int64_t pitch, int64_t row0,
                         int64_t stride, uint8_t value, int ilv, hipStream_t s);
// Block rows of a ragged board (gol_formats.hip): aligned rows of ring_pitch(W, torus) words in layout ilv (1 or 2).
// Torus: ring rows, position u = cell (u - 64) mod W; bounded: position u = cell u, zero past W.  Pack / unpack
// against the byte board, and (torus) the per-pass refresh of the ring's two copies.
int64_t ring_pitch(int64_t W, bool torus);
hipError_t launch_pack_ring(const uint8_t* cells, uint32_t* words, int64_t W, int64_t H, int ilv, bool torus,
                            hipStream_t s);
hipError_t launch_unpack_ring(const uint32_t* words, uint8_t* cells, int64_t W, int64_t H, int ilv, bool torus,
                              hipStream_t s);
hipError_t launch_ring_refresh(uint32_t* words, int64_t W, int64_t H, int ilv, hipStream_t s);
hipError_t launch_region(const void* board, int ilv, int64_t W, int64_t pitch, int64_t x0, int64_t y0, int64_t w,
                         int64_t h, uint8_t* out, hipStream_t s);
hipError_t launch_bytes_render(const uint8_t* cells, uint8_t* out, int64_t W, int64_t H, int64_t stride,
                               uint8_t value, hipStream_t s);
hipError_t launch_splitmix_packed(uint32_t* words, int64_t wpr, int64_t rows, int64_t pitch, int64_t row0,
                                  int64_t gy0, uint64_t seed, int ilv, hipStream_t s);
hipError_t launch_splitmix_bytes(uint8_t* cells, int64_t W, int64_t H, uint64_t seed, hipStream_t s);
hipError_t launch_popcount_packed(const uint32_t* words, int64_t wpr, int64_t rows, int64_t pitch, int64_t row0,
                                  unsigned long long* acc, hipStream_t s);
hipError_t launch_popcount_bytes(const uint8_t* cells, int64_t n, unsigned long long* acc, hipStream_t s);
hipError_t launch_hash_packed(const uint32_t* words, int64_t W, int64_t rows, int64_t pitch, int64_t row0,
                              int64_t gy0, int ilv, unsigned long long* acc, hipStream_t s);
hipError_t launch_hash_bytes(const uint8_t* cells, int64_t W, int64_t H, unsigned long long* acc, hipStream_t s);
// canonical snapshot rows (ceil(W/64) uint64 per row); ilv = 0: byte board
hipError_t launch_export_canonical(const void* board, int64_t W, int64_t rows, int64_t pitch, int64_t row0, int ilv,
                                   uint64_t* out, hipStream_t s);
hipError_t launch_import_canonical(const uint64_t* in, int64_t W, int64_t rows, int64_t pitch, int64_t row0, int ilv,
                                   void* board, hipStream_t s);
hipError_t launch_set_points(void* board, int ilv, int64_t W, int64_t pitch, const int64_t* xy, int64_t n,
                             hipStream_t s);

// ---- gol_resident.hip: whole board in one workgroup's LDS, all generations in one launch
bool resident_packed_fits(int64_t W, int64_t H);  // ilv = 1 layout
bool resident_bytes_fits(int64_t W, int64_t H);
// threads: 1024 (default) or 256 (board option "resident_threads")
hipError_t launch_resident_packed(const uint32_t* src, uint32_t* dst, int64_t W, int64_t H, int64_t pitch,
                                  int64_t gens, bool bounded, hipStream_t s, int threads = 1024);
hipError_t launch_resident_bytes(const uint8_t* src, uint8_t* dst, int64_t W, int64_t H, int64_t gens, bool bounded,
                                 hipStream_t s, int threads = 1024);

// ---- gol_coop.hip: one workgroup per CU owning a band of rows in registers, k generations per neighbour
// hand-off (boards up to 8192 wide, ilv 1 or ilv = coop_m); the result lands in dst
constexpr int kCoopDefaultK = 8;  // generations per hand-off unless the board's "coop_k" option or tblock_k says less
int coop_m(int64_t nw);  // words per lane for rows of nw words (0: too wide for the pass)
// min_rows: rows per wave at least (board option "coop_r", 1 by default)
bool coop_plan(int64_t W, int64_t H, int k, int* nwg, int* B, int* R, int min_rows = 1);
int64_t coop_xch_words(int64_t W, int nwg, int k);  // exchange buffer the pass needs
// gens <= 65535 per launch; epoch (1..65535) tags this launch's hand-off granules (clear xch before reusing one).
// ragged_w > 0: a ragged board (width ragged_w, not a multiple of 32) packed into whole-word scratch rows of W cells
// (launch_pack_ragged), ilv 1; 0: a packed board of width W.
// poll_delay: s_sleep 1 periods before a hand-off's first poll (8); spin_limit: polls before a wait gives up and
// sets *err (0 = the default, ~2 s); min_rows as for coop_plan.
struct CoopTuning {
    int min_rows = 1;
    int poll_delay = 8;
    unsigned spin_limit = 0;
    bool plain_launch = false;  // hipLaunchKernel instead of hipLaunchCooperativeKernel (the grid fits by construction)
};
hipError_t launch_coop_pass(const uint32_t* src, uint32_t* dst, int64_t W, int64_t H, int64_t pitch, int ilv, int k,
                            int64_t gens, bool bounded, unsigned epoch, int* err, uint32_t* xch, int64_t xch_words,
                            hipStream_t s, int64_t ragged_w = 0, const CoopTuning& tune = CoopTuning());

// A persistent launch whose workgroups wait on each other (the cooperative and rows-on-lanes passes): every
// workgroup must be resident at once.  cooperative: hipLaunchCooperativeKernel; else hipLaunchKernel after the same
// check against the occupancy API (hipErrorCooperativeLaunchTooLarge when the grid cannot be resident).  The plain
// launch is the default (board option "coop_launch"): the runtime's cooperative-launch state is torn down at process
// exit after a profiler's (rocprofv3 --kernel-trace) and faulted there (DESIGN.md 6 "Exit under rocprofv3").
// Persistent launches of all boards are serialised per device (each waits on the device's previous one), so two
// such grids are never resident together.
hipError_t launch_persistent(const void* fn, unsigned grid, unsigned threads, void** args, size_t lds, hipStream_t s,
                             bool cooperative);
// Workgroups of (fn, threads, lds) the current device holds at once (occupancy API x CUs; cached per device), -1 on
// error; CUs of the current device (cached per device, 0 without one); the dynamic-LDS attribute once per
// (device, kernel).
int64_t persistent_capacity(const void* fn, unsigned threads, size_t lds);
int device_cus();
hipError_t set_max_dynamic_lds(const void* fn, int bytes);

// ---- gol_lanes.hip: rows-on-lanes band pass (a wave owns all rows of a band window of 64 (m - 1) columns and
// steps it k generations alone), packed boards of any interleave, W a multiple of 64 (m - 1), k <= 16
struct LanesPlan {
    int m = 0;     // words per lane and half-row (5, 9 or 17)
    int nx = 0;    // windows per band (waves per workgroup)
    int nb = 0;    // bands (workgroups)
    int bmax = 0;  // rows of the tallest band
};
// m_opt: 0 = by width (3 up to 1024 columns, else 9 when W % 512 == 0, else 5), or 3 / 5 / 9 / 17
bool lanes_plan(int64_t W, int64_t H, int k, int m_opt, LanesPlan* out);
int64_t lanes_xch_words(const LanesPlan& p, int k);
// The plan's bands can all be resident at once on the current device (a tall narrow board plans more
// bands than the device holds; such a board takes the cooperative or the streaming pass instead)
bool lanes_fits(int64_t W, int64_t H, int k, int m_opt, int ilv, bool bounded);
// as launch_coop_pass (gens <= 65535 per launch, epoch-tagged granules in xch, *err on a timed-out wait)
hipError_t launch_lanes_pass(const uint32_t* src, uint32_t* dst, int64_t W, int64_t H, int64_t pitch, int ilv, int k,
                             int64_t gens, bool bounded, unsigned epoch, int* err, uint32_t* xch, int64_t xch_words,
                             hipStream_t s, int m_opt, const CoopTuning& tune);

// ---- gol_wave.hip: whole board in one wavefront's registers (W <= 128, H <= 256), all generations in one launch
int wave_resident_rpl(int64_t W, int64_t H);  // rows per lane, 0 = the board does not fit
hipError_t launch_wave_resident(const void* src, void* dst, int64_t W, int64_t H, int64_t pitch, int64_t gens,
                                bool bounded, bool bytes, hipStream_t s);

}  // namespace gol
