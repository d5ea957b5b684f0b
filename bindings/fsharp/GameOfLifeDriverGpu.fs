// GameOfLifeDriverGpu.fs -- drop-in for GameOfLife/GameOfLife/GameOfLifeDriver.fs:13-41: `run()` keeps its
// signature; the W*H cell agents are replaced by one GolNative.Board.  Uses the unchanged render agent
// (GameOfLifeUI.fs) and types (GameOfLifeLogic.fs).  Not compiled here; see INTEGRATION.md.
module GameOfLifeDriverGpu

open System
open GameOfLifeLogic
open GameOfLifeUI

let run () : IDisposable =
    let updateAgent = updateAgent ()                         // GameOfLifeUI.fs:13, unchanged
    let board = new GolNative.Board(grid.Width, grid.Height, GolNative.Boundary.Torus)
    board.Seed(int DateTime.Now.Ticks, GolNative.InitMode.DotNetMod2)   // L9-11,16-19: same RNG, same order

    let updateView () =                                      // L32-34: one tick = one generation
        updateAgent.Post UpdateView.Reset
        board.Step 1L
        let cells = board.GetCells()                         // cells.[x + y*W]
        applyGrid (fun x y ->                                // GameOfLifeLogic.fs:13-15 order
            updateAgent.Post(Update(cells.[x + y * grid.Width] = 1uy, { x = x; y = y })))

    updateAgent.Start()
    let timer = new System.Timers.Timer(float Environment.ProcessorCount * 70.)   // L38
    let sub = timer.Elapsed.Subscribe(fun _ -> updateView ())                       // L39
    timer.Start()                                                                   // L40
    { new IDisposable with
        member _.Dispose() = sub.Dispose(); timer.Dispose(); (board :> IDisposable).Dispose() }
