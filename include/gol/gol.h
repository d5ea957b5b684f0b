/*
 * gol.h -- C ABI of the MI355X Game of Life engine (libgol_hip.so).
 *
 * Drop-in boundary for the reference's hot path: the per-cell actors of
 *   GameOfLife/GameOfLife/GameOfLifeLogic.fs:39-71   (MailboxProcessor cell, `createCell`)
 *   GameOfLife/GameOfLifeAkka/GameofLife.fs:88-138   (Akka `CellAkka`, `ICell.Send`)
 * and the dictionary of them built by the driver (GameOfLifeDriver.fs:16-30, GameofLife.fs:148-163).
 * One board handle replaces the W*H cell actors; `gol_step(b, 1)` replaces one `updateView()` tick
 * (GameOfLifeDriver.fs:32-34); `gol_render_gray8` / `gol_get_cells` replace the W*H `Update` posts
 * consumed by the render agent (GameOfLifeUI.fs:21-31).  The F# P/Invoke declarations that bind each
 * entry point are in INTEGRATION.md.
 *
 * Conventions: cdecl, plain pointers, int64_t sizes.  Every function returns 0 (GOL_OK) or a negative
 * GOL_ERR_* code; gol_last_error() returns a thread-local message for the last failure on the calling
 * thread.  No C++ exception crosses this ABI.  Host buffers are borrowed for the duration of the call
 * only (P/Invoke pins blittable byte[] for the call).  Each board handle is serialised by an internal
 * mutex (the reference's timer can re-enter updateView, GameOfLifeDriver.fs:38-40); separate handles are
 * independent.  Cell layout for host buffers: one byte per cell, index x + y*width, nonzero = alive
 * (GameOfLifeUI.fs:24-28 pixel order).
 */
#ifndef GOL_GOL_H
#define GOL_GOL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GOL_OK 0
#define GOL_ERR_INVALID -1     /* bad argument, size or geometry */
#define GOL_ERR_HIP -2         /* HIP runtime / kernel launch failure */
#define GOL_ERR_OOM -3         /* device allocation failed */
#define GOL_ERR_UNSUPPORTED -4 /* valid request this build does not implement */
#define GOL_ERR_NO_DEVICE -5   /* no usable gfx950 device */

enum { GOL_TORUS = 0, GOL_BOUNDED = 1 };
/* gol_seed_dotnet modes */
enum {
    GOL_INIT_DOTNET_MOD2 = 0, /* GameOfLifeDriver.fs:9-11,16-19: x outer, y inner, Random.Next() % 2 = 0 */
    GOL_INIT_DOTNET_NEXT2 = 1 /* Script.fsx:25-27: Array2D.init (x outer), Random.Next 2 = 0 */
};

typedef struct gol_board gol_board; /* opaque; library-owned */

/* Replaces `cells = seq { for x .. for y .. createCell ... } |> dict` (GameOfLifeDriver.fs:16-19) and the
 * neighbour wiring (L21-30).  width/height >= 3 (smaller tori alias neighbours: the reference's
 * Dictionary never reaches 8 keys and the board freezes, GameOfLifeLogic.fs:58 -- rejected here).
 * boundary: GOL_TORUS (actors, GameOfLifeDriver.fs:25) or GOL_BOUNDED (Script.fsx:11).
 * num_gpus: 1 = one board on the calling thread's current device.  N > 1 = row strips on devices
 *           0..N-1 of THIS process (the reference host is one process, GameOfLifeDriver.fs:13-41): strip r
 *           owns rows [H*r/N, H*(r+1)/N); every pass moves k halo rows between neighbouring strips while the
 *           interior rows compute.  Halo transport: peer copies (hipMemcpyPeerAsync, xGMI between GPUs) by
 *           default; RCCL send/recv on request (gol_set_option "transport" = 2, distinct devices only;
 *           gol_transport reports which one runs).  Needs width % 32 == 0.  Bit-identical to num_gpus = 1.
 *           (One process per GPU instead: gol_strip_* below.)
 * tblock_k: upper bound on the generations fused per kernel pass (0 = the engine's default for the
 *           board, gol_layout / gol_info report it):
 *             packed boards below 2^25 cells: ilv 1, k = 8 (latency-bound: the single-wave pass takes boards up
 *               to 128 x 256), except single boards the cooperative pass takes (2^17 < cells <=
 *               2^26, 4096 or 8192 wide): ilv 2 / 4 (that pass's words per lane) and k = 16 / 8, of
 *               which it hands off every min(k, 8) generations;
 *             packed boards of 2^25 .. 2^29 cells, width % 64 == 0: ilv 2, k = 16;
 *             boards from 2^30 cells per part, width % 128 == 0 and >= 7936 (torus) or 8192 (bounded): ilv 4,
 *               k = 32 -- the level-pipelined pass (k = 16 / 32 at ilv 4 is that pass);
 *             other packed boards from 2^29 cells, width % 64 == 0: ilv 2, k = 12 -- torus and bounded alike
 *               (bounded boards ran k = 16 until round 3), single board or strips;
 *             other packed widths from 2^25 cells: ilv 1, k = 32;
 *             byte boards (width % 32 != 0, ilv 0) below 3 * 2^26 cells: k = 8 below 2^25 cells, 16 below 2^27,
 *               24 above (the ilv-1 scratch rows they stream as);
 *             byte boards from 3 * 2^26 cells: the rules above for the block rows they stream as (DESIGN.md 4.1
 *               "Ragged rows": 2 * ceil((W + 128) / 64) words per ring row on a torus, 2 * ceil(W / 64) when
 *               bounded; ilv 2 k = 16 below 2^29 of those cells, k = 12 above);
 *           else one of 1,2,4,6,8,12,16,24,32 -- the engine uses the deepest supported depth <= tblock_k (a
 *           depth the automatic ilv 4 does not run, 12 or 24, selects ilv 2 instead).
 *           A multi-part board's halo depth (gol_part_info ghost) is the deepest supported k <= tblock_k that
 *           fits its thinnest strip.
 * The initial board is all dead. */
int gol_create(int64_t width, int64_t height, int boundary, int num_gpus, int tblock_k, gol_board** out);
/* As gol_create with an explicit packed layout: ilv = 0 (auto, gol_default_ilv) or 1, 2, 4 words per
 * interleaved block (width must be a multiple of 32*ilv). */
int gol_create_ex(int64_t width, int64_t height, int boundary, int num_gpus, int tblock_k, int ilv,
                  gol_board** out);
/* As gol_create_ex with num_gpus = ndevices and strip r placed on devices[r] (a device may repeat, e.g.
 * to run the multi-strip protocol on one GPU). */
int gol_create_multi(int64_t width, int64_t height, int boundary, const int* devices, int ndevices, int tblock_k,
                     int ilv, gol_board** out);
/* Row strips of a board (1 unless created with num_gpus > 1) and where strip `part` lives: its device,
 * first global row, owned rows and halo depth (ghost rows per side; 0 for a single board). */
int gol_num_parts(gol_board* b, int* n);
int gol_part_info(gol_board* b, int part, int* device, int64_t* y0, int64_t* rows, int64_t* ghost);
/* How a multi-part board moves its halo rows: peer copies (the default) or RCCL send/recv (ncclCommInitAll over
 * the parts' devices, xGMI) once gol_set_option(b, "transport", GOL_TRANSPORT_RCCL) succeeded -- it fails with
 * GOL_ERR_UNSUPPORTED when a device repeats (RCCL refuses two ranks on one GPU) or RCCL is unavailable, and the
 * board keeps peer copies.  A single board has none.  note (may be NULL, >= 256 bytes): a description. */
enum { GOL_TRANSPORT_NONE = 0, GOL_TRANSPORT_PEER = 1, GOL_TRANSPORT_RCCL = 2 };
int gol_transport(gol_board* b, int* transport, char* note, int64_t note_len);
int gol_destroy(gol_board* b);

/* Board I/O: cells[x + y*width], len == width*height.  Replaces createCell's `alive` argument
 * (GameOfLifeLogic.fs:39) and, on readback, the per-cell Update(alive, location) stream (L64). */
int gol_set_cells(gol_board* b, const uint8_t* cells, int64_t len);
int gol_get_cells(gol_board* b, uint8_t* cells, int64_t len);
/* Read a window (x, y, w, h) of the board (no wrap; must lie inside): out[i + j*w] = cell (x+i, y+j). */
int gol_get_region(gol_board* b, int64_t x, int64_t y, int64_t w, int64_t h, uint8_t* out);

/* Seeding.  gol_seed_dotnet restates .NET Framework System.Random(seed) exactly as the reference uses it
 * (GameOfLifeDriver.fs:9-11 with an explicit seed instead of DateTime.Now.Ticks).  gol_seed_splitmix is
 * the build-owned device-side init for large boards.  gol_place_rle ORs a Life RLE pattern
 * with its top-left at (x, y), wrapped modulo the board. */
int gol_seed_dotnet(gol_board* b, int32_t seed, int mode);
/* Board snapshot (save / restore, SURVEY 8f "board save/load") in the canonical bit-packed layout the
 * hash is defined on, independent of the board's internal layout and GPU count: row y is ceil(width/64)
 * little-endian uint64 words, bit i of word j = cell (64j + i, y), bits past the width zero;
 * len = height * ceil(width/64).  A snapshot taken from any board loads into any board of the same size.
 * gol_load_packed resets the generation counter (like gol_set_cells). */
int gol_save_packed(gol_board* b, uint64_t* words, int64_t len);
int gol_load_packed(gol_board* b, const uint64_t* words, int64_t len);
int gol_seed_splitmix(gol_board* b, uint64_t seed);
int gol_place_rle(gol_board* b, const char* rle, int64_t x, int64_t y);
int gol_clear(gol_board* b);

/* Advance `generations` synchronous B3/S23 generations (GameOfLifeLogic.fs:47-66 under the Reset->State
 * phase barrier).  Asynchronous with respect to the host; any readback synchronises (and reports a failed
 * cooperative pass: the board is then invalid until overwritten).  Small and mid-size boards run the whole call
 * as one launch (single-wave, cooperative or LDS-resident pass: DESIGN.md 4.3-4.5; gol_set_option moves the
 * cut-overs); results are identical either way.  A board whose width is not a multiple of 32 runs calls of several
 * generations on whole-word scratch rows (DESIGN.md 4.1 "Ragged rows") and keeps its state there until another
 * call reads or replaces the cells. */
int gol_step(gol_board* b, int64_t generations);
int gol_generation(gol_board* b, int64_t* out);
int gol_synchronize(gol_board* b);
/* Profiling: gol_step between two HIP timing events on the board's stream, then synchronise; *elapsed_us = the
 * device time of the call (multi-part boards: each part times its own compute stream, the longest is reported).
 * Lets a host without any other GPU runtime (the F# driver) time the engine under the HIP runtime it loads. */
int gol_step_timed(gol_board* b, int64_t generations, double* elapsed_us);

/* Replaces the render agent's pixel fill (GameOfLifeUI.fs:24-28; GameofLife.fs:53-57; Script.fsx:33-35):
 * pixels[x + y*stride] = alive ? alive_value : 0, stride >= width, buffer >= stride*height bytes. */
int gol_render_gray8(gol_board* b, uint8_t* pixels, int64_t stride, uint8_t alive_value);

/* Observables for parity checks. */
int gol_population(gol_board* b, int64_t* out);
int gol_hash(gol_board* b, uint64_t* out); /* canonical 64-bit board hash */

/* Introspection: width, height, boundary, tblock_k, packed (1 = bit-packed path, 0 = byte path). */
int gol_info(gol_board* b, int64_t* width, int64_t* height, int* boundary, int* tblock_k, int* packed);
/* Packed layout of the board: ilv = words per interleaved block (1, 2, 4; 0 = byte board), pitch in words. */
int gol_layout(gol_board* b, int* ilv, int64_t* pitch);
/* Layout / depth the engine picks for a large board of this width (0 if the width is not a multiple of
 * 32; boards below 2^25 cells use ilv 1, see gol_create), the default temporal-block depth for a layout
 * on a large board, and whether the step kernel supports depth k for a layout. */
int gol_default_ilv(int64_t width);
/* HIP devices visible to this process (0 and GOL_OK when there is none). */
int gol_device_count(int* n);
int gol_default_tblock(int ilv);
int gol_supported_k(int k, int ilv);
/* The layout and depth the engine picks for a board or row strip of `rows` rows (gol_create uses the same rule):
 * boards of >= 2^30 cells at least 7936 cells wide on a torus, 8192 bounded (width % 128 == 0) run the
 * level-pipelined pass, ilv 4 and K = 32; others as gol_default_ilv / gol_default_tblock.  k = 16 / 32
 * at ilv 4 is that pass (gol_strip_step refuses it on narrower strips). */
int gol_default_layout(int64_t width, int64_t rows, int boundary, int* ilv, int* tblock_k);
/* The HIP stream the board's kernels run on (hipStream_t), for event timing by a caller (multi-GPU
 * boards: strip 0's compute stream, which every pass joins at its end). */
int gol_stream(gol_board* b, void** stream);

/* Profiling: advance the board by ONE pass of its temporal depth with HIP timing events and report, per
 * row strip (n = gol_num_parts), the microseconds from the pass start to the end of the interior launch
 * (interior_us), to the release of the edge-band stream once the neighbours' halo rows have landed
 * (wait_us: the edge-band wait) and to the end of the edge bands (edge_us).  A single board times one
 * streaming pass and reports it in interior_us and edge_us and 0 in wait_us; a single board whose gol_step
 * runs another pass (single-wave, cooperative, LDS-resident) returns GOL_ERR_UNSUPPORTED.  Counts toward
 * gol_generation. */
int gol_pass_timing(gol_board* b, int n, double* interior_us, double* wait_us, double* edge_us);

/* Per-board path and tuning options (the library reads no environment variable).  Names, defaults first:
 *   "coop" 1 | 0                 cooperative register-band pass for mid-size boards
 *   "coop_k" 0 | 1..64           generations per band hand-off (0: min(tblock_k, 8))
 *   "coop_max_cells" 2^26        largest board that pass takes
 *   "resident_max_cells" -1 | n  LDS-resident pass cut-over (-1: 2^17 packed cells, off for byte boards; 0: off)
 *   "wave_resident" 1 | 0        single-wave pass for boards up to 128 x 256
 *   "split" 0 | n | -1           streaming pass: the oldest wave's share of a SIMD group segment in 1/65536
 *                                (0: the measured default, -1: no split)
 *   "split2" 0 | n               streaming pass, three waves per SIMD group: the middle wave's share of the two
 *                                younger waves' rows in 1/65536 (0: the measured default)
 *   "seg_rows" 0 | n             streaming pass: rows per wave segment (0: planned)
 *   "seam" 0 | -1                streaming pass on a torus: seam strips where they apply (-1: halo-lane strips)
 *   "transport" 1 | 2            multi-part boards: halo rows by peer copies (1) or RCCL (2, distinct devices;
 *                                GOL_ERR_UNSUPPORTED otherwise); GOL_ERR_UNSUPPORTED on a single board
 *   ("split", "split2", "seg_rows" and "seam" apply to every strip launch of a multi-part board as well)
 *   "ragged_ring" 1 | 2 | 0      ragged boards on the streaming pass as block rows in the aligned layouts (torus: ring
 *                                rows; bounded: column-masked rows) from 3 * 2^26 cells (1), on every size (2), or
 *                                never (0: ilv-1 rows)
 *   "ragged_stream" 1 | 0        boards of any width beyond the cooperative pass: the streaming pass on scratch
 *                                words (0: the per-generation byte step)
 *   "coop_poll_delay" -1 | 0..4096  s_sleep periods before a hand-off's first poll (-1: on the cooperative pass 0 for
 *                                4096-cell rows, 4 for narrower ones, 24 for every width above 4096; 8 on the rows-on-lanes pass)
 *   "lanes" 2 | 1 | 0            rows-on-lanes band pass in place of the cooperative one (packed single boards whose
 *                                width splits into 128/256/512/1024-column windows, coop_k <= 10, calls of >= 2 k
 *                                generations, every band resident at once): 2 = on the sizes it
 *                                measured faster (rows of <= 1024 cells), 1 = wherever it
 *                                applies, 0 = never
 *   "lanes_m" 0 | 3 | 5 | 9 | 17 its words per lane and half-row (0: 3 up to 1024 columns, else 9 when W % 512 == 0)
 * Unknown names and out-of-range values return GOL_ERR_INVALID.  Results are bit-identical for every setting.
 * (Test and A/B knobs -- spin limits, tag epochs, launch API -- are not board options: they live behind
 * gol_debug_set_option in the library's internal header csrc/gol_debug.h.)
 * The persistent passes (cooperative, rows-on-lanes) of all boards of a process are serialised per device, so two
 * handles stepping at once from two threads never split the CUs between two such grids.  The serialisation is per
 * PROCESS: a second process stepping a mid-size board on the same GPU at the same time can hold CUs a persistent grid
 * needs.  Its bands then wait out the spin limit (~2 s), the call's board is left wrong, and the next
 * gol_synchronize or readback returns GOL_ERR_HIP with gol_last_error() naming that cause ("a band hand-off timed
 * out -- the pass could not get every CU at once ...").  Set "coop" 0 on boards that share a GPU with other
 * processes: every generation then runs on the ordinary (non-persistent) passes. */
int gol_set_option(gol_board* b, const char* name, int64_t value);
int gol_get_option(gol_board* b, const char* name, int64_t* value);

const char* gol_last_error(void);
const char* gol_version(void);
/* 1 if a device reporting this hipDeviceProp_t::gcnArchName ("gfx950", "gfx950:sramecc+:xnack-") runs this
 * build, else 0.  gol_create returns GOL_ERR_NO_DEVICE for a board on any other device. */
int gol_arch_supported(const char* gcn_arch_name);

/* ------------------------------------------------------------------------------------------------
 * Row-strip entry points for multi-GPU runs (one process per GPU; the caller owns device memory and
 * does the halo exchange, e.g. RCCL send/recv).  A strip buffer holds `ghost` halo rows, then `rows`
 * owned rows (global rows [y0, y0+rows)), then `ghost` halo rows; each buffer row is `pitch` 32-bit
 * words, of which the first width/32 are the board row in the interleaved layout `ilv`:
 *     row = blocks of ilv words; in block k, word j bit b = cell x = 32*ilv*k + j + ilv*b
 * (ilv = 1: bit b of word w = cell 32w + b).  width must be a multiple of 32*ilv, pitch of ilv.  With world size 1 a strip may instead set wrap_rows = 1, ghost = 0,
 * rows = height: torus rows then wrap inside the buffer (the single-GPU board layout).
 * `stream` is a hipStream_t (NULL = default stream).  All calls are asynchronous. */
typedef struct gol_strip {
    int64_t width;    /* global board width (cells) */
    int64_t height;   /* global board height (rows) */
    int64_t y0;       /* global row of owned row 0 */
    int64_t rows;     /* owned rows */
    int64_t ghost;    /* halo rows above and below (>= k for a k-generation pass unless wrap_rows) */
    int64_t pitch;    /* words per buffer row (>= width/32) */
    int32_t boundary; /* GOL_TORUS | GOL_BOUNDED */
    int32_t wrap_rows;
    int32_t ilv;      /* words per interleaved block: 1, 2 or 4 (gol_default_ilv) */
    int32_t spare_waves; /* waves gol_strip_step leaves free for concurrent work on other streams (e.g. the
                            halo bands of the same pass); 0 = fill the device */
} gol_strip;

/* k generations over owned rows [out_begin, out_end) from src to dst (distinct buffers, same geometry).
 * Reads rows [out_begin-k, out_end+k); with wrap_rows = 0 those must lie in [-ghost, rows+ghost). */
int gol_strip_step(const gol_strip* s, const uint32_t* src, uint32_t* dst, int k, int64_t out_begin,
                   int64_t out_end, void* stream);
int gol_strip_seed_splitmix(const gol_strip* s, uint32_t* buf, uint64_t seed, void* stream);
/* cells: host or device bytes of the owned rows, cells[x + r*width] (r = owned row) */
int gol_strip_pack(const gol_strip* s, const uint8_t* dev_cells, uint32_t* buf, void* stream);
int gol_strip_unpack(const gol_strip* s, const uint32_t* buf, uint8_t* dev_cells, int64_t stride, uint8_t value,
                     void* stream);
/* Add this strip's population / canonical-hash partial sum into *dev_acc (device uint64). */
int gol_strip_population(const gol_strip* s, const uint32_t* buf, uint64_t* dev_acc, void* stream);
int gol_strip_hash_partial(const gol_strip* s, const uint32_t* buf, uint64_t* dev_acc, void* stream);
/* Combine the (wrapping) sum of every strip's partial into the canonical board hash. */
uint64_t gol_hash_finalize(uint64_t partial_sum, int64_t width, int64_t height);
/* The halo messages of one pass of a multi-part board (one process, gol_create num_gpus > 1), in the order each
 * part issues them -- the plan both transports execute: op 0 = send, 1 = recv; rows are buffer rows of the part
 * (0 = the first of `ghost` halo rows).  Host-only (no device needed): tests check that every receive gets the
 * rows the topology gives it under RCCL's in-order pairing. */
typedef struct gol_xfer {
    int32_t part, op, peer, pad;
    int64_t row, nrows;
} gol_xfer;
int gol_exchange_plan(int64_t height, int boundary, int nparts, int64_t ghost, int k, gol_xfer* ops, int64_t max_ops,
                      int64_t* n_ops);
/* Number of wavefront column strips / rows per segment the step kernel uses (for roofline accounting). */
int gol_strip_plan(const gol_strip* s, int k, int64_t out_begin, int64_t out_end, int64_t* waves,
                   int64_t* seg_rows);
/* The whole plan (n >= 8): plan[0..7] = column strips, row segments, rows per segment, seam geometry (1 / 0),
 * remainder blocks per row, remainder sub-strips per wave, packed remainder segments (segments 1 .. plan[6] share
 * remainder waves), remainder units; with n >= 10 also plan[8..9] = the SIMD groups' split and second split (1/65536
 * units, 0 = unsplit / geometric).  Planned for the current device's resident waves (4096 without a device):
 * tests/test_cpu_host.py walks it to check that no wave reads outside its buffer. */
int gol_strip_plan_ex(const gol_strip* s, int k, int64_t out_begin, int64_t out_end, int64_t* plan, int64_t n);

#ifdef __cplusplus
}
#endif
#endif /* GOL_GOL_H */
