// GameOfLifeAkkaGpu.fs -- drop-in for the Akka project's driver, GameOfLife/GameOfLifeAkka/GameofLife.fs:140-174
// (`GameOfLifeAgent.run`).  `run()` keeps its shape (returns the timer subscription as an IDisposable); the
// actor system and the W*H `CellAkka` actors (L146-163) are replaced by one GolNative.Board, and each 200 ms
// tick (L171) advances it one generation and feeds the unchanged render agent (`updateAgent`, L42-64).
// Compiled into the Akka project after GameofLife.fs and GolNative.fs; not compiled here (no dotnet), see
// INTEGRATION.md.
namespace GameOfLife

open System
open GameOfLife.GameOfLifeAgent

module GameOfLifeAkkaGpu =

    let run () : IDisposable =
        let updateAgent = updateAgent ()                                   // L165 (L42-64 unchanged)
        let board = new GolNative.Board(grid.Width, grid.Height, GolNative.Boundary.Torus)
        // L140-142, L148-152: one Random(int DateTime.Now.Ticks), Next() % 2 = 0, drawn x outer / y inner
        // while `dict` materialises the cells -- gol_seed_dotnet restates exactly that order
        board.Seed(int DateTime.Now.Ticks, GolNative.InitMode.DotNetMod2)

        let updateView () =                                                 // L165-167: one tick = one generation
            updateAgent.Post(UpdateView.Reset)
            board.Step 1L
            let cells = board.GetCells()                                    // cells.[x + y*W]
            applyGrid (fun x y ->                                           // L34-36 order, Update of bool * Location
                updateAgent.Post(Update(cells.[x + y * grid.Width] = 1uy, { x = x; y = y })))

        do updateAgent.Start()                                              // L169
        let timer = new System.Timers.Timer(200.)                           // L171
        let sub = timer.Elapsed |> Observable.subscribe (fun _ -> updateView ())   // L172
        timer.Start()                                                       // L173
        { new IDisposable with
            member _.Dispose() =
                sub.Dispose()
                timer.Dispose()
                (board :> IDisposable).Dispose() }
