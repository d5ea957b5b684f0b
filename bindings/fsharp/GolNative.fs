// GolNative.fs -- F# P/Invoke binding of libgol_hip.so (include/gol/gol.h), for the reference's
// GameOfLife / GameOfLifeAkka projects (add before GameOfLifeDriver.fs in GameOfLife.fsproj:59-65).
// Not compiled in this repository (no dotnet in the build image); the same entry points are exercised
// through ctypes by tests/. See INTEGRATION.md.
module GolNative

open System
open System.Runtime.InteropServices

[<Literal>]
let Lib = "gol_hip"   // libgol_hip.so (Linux) / gol_hip.dll; ships next to the executable

type Boundary = Torus = 0 | Bounded = 1          // GameOfLifeDriver.fs:25 | Script.fsx:11
type InitMode = DotNetMod2 = 0 | DotNetNext2 = 1 // GameOfLifeDriver.fs:9-11,16-19 | Script.fsx:25-27

[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int gol_create(int64 width, int64 height, int boundary, int numGpus, int tblockK, nativeint& board)
[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int gol_destroy(nativeint board)
[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int gol_set_cells(nativeint board, byte[] cells, int64 len)        // cells.[x + y*W], 0/1
[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int gol_get_cells(nativeint board, byte[] cells, int64 len)
[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int gol_seed_dotnet(nativeint board, int seed, int mode)
[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int gol_step(nativeint board, int64 generations)
[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int gol_render_gray8(nativeint board, byte[] pixels, int64 stride, byte aliveValue)
[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int gol_save_packed(nativeint board, uint64[] words, int64 len)   // canonical snapshot, H*ceil(W/64)
[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int gol_load_packed(nativeint board, uint64[] words, int64 len)
[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int gol_population(nativeint board, int64& out)
[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int gol_hash(nativeint board, uint64& out)
[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int gol_synchronize(nativeint board)
[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int gol_set_option(nativeint board, [<MarshalAs(UnmanagedType.LPStr)>] string name, int64 value)
[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int gol_transport(nativeint board, int& transport, System.Text.StringBuilder note, int64 noteLen)
[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int gol_step_timed(nativeint board, int64 generations, double& elapsedUs)
[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern int gol_device_count(int& n)
[<DllImport(Lib, CallingConvention = CallingConvention.Cdecl)>]
extern nativeint gol_last_error()

let check (what: string) rc =
    if rc <> 0 then
        failwithf "%s failed (%d): %s" what rc (Marshal.PtrToStringAnsi(gol_last_error()))

/// One board in HBM: replaces the W*H cell agents (GameOfLifeLogic.fs:39-71).  numGpus > 1 spreads it
/// over GPUs 0..numGpus-1 of this process as row strips (bit-identical; width must be a multiple of 32).
type Board(width: int, height: int, boundary: Boundary, ?numGpus: int) =
    let mutable h = 0n
    do check "gol_create" (gol_create(int64 width, int64 height, int boundary, defaultArg numGpus 1, 0, &h))
    member _.Seed(seed: int, mode: InitMode) = check "gol_seed_dotnet" (gol_seed_dotnet(h, seed, int mode))
    member _.Step(generations: int64) = check "gol_step" (gol_step(h, generations))
    member _.GetCells() =
        let a = Array.zeroCreate<byte> (width * height)
        check "gol_get_cells" (gol_get_cells(h, a, int64 a.Length)); a
    member _.Render(pixels: byte[], alive: byte) =
        check "gol_render_gray8" (gol_render_gray8(h, pixels, int64 width, alive))
    member _.Save() =   // 1 bit per cell, layout- and GPU-count-independent
        let w = Array.zeroCreate<uint64> (height * ((width + 63) / 64))
        check "gol_save_packed" (gol_save_packed(h, w, int64 w.Length)); w
    member _.Load(words: uint64[]) = check "gol_load_packed" (gol_load_packed(h, words, int64 words.Length))
    /// gol_step timed by the library's own HIP events (device microseconds of the call): the host's own figure,
    /// under the HIP runtime the library links -- no other GPU runtime in the F# process.
    member _.StepTimed(generations: int64) =
        let mutable us = 0.0
        check "gol_step_timed" (gol_step_timed(h, generations, &us)); us
    /// Wait for the board's work; reports a failed cooperative pass (GOL_ERR_HIP) like every readback.
    member _.Synchronize() = check "gol_synchronize" (gol_synchronize h)
    /// Path / tuning option (gol.h lists the names, e.g. "coop" 0); results are bit-identical for every setting.
    member this.SetOption(name: string, value: int64) =
        check "gol_set_option" (gol_set_option(h, name, value)); this
    /// Halo transport of a multi-GPU board: 0 none (one part), 1 peer copies (the default), 2 RCCL (after
    /// SetOption("transport", 2L), one strip per GPU); with a description.
    member _.Transport() =
        let mutable t = 0
        let note = System.Text.StringBuilder(256)
        check "gol_transport" (gol_transport(h, &t, note, int64 note.Capacity)); (t, note.ToString())
    interface IDisposable with
        member _.Dispose() = if h <> 0n then (gol_destroy h |> ignore; h <- 0n)
