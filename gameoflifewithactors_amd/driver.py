"""Headless mirror of the reference driver and render agent, running on the HIP engine.

* ``run()``          -- ``GameOfLife/GameOfLife/GameOfLifeDriver.fs:13-41`` (Akka: ``GameofLife.fs:144-174``)
* ``UpdateAgent``    -- ``GameOfLifeUI.fs:13-35`` without WPF: it collects ``Update`` messages and
                        fills the Gray8 ``pixels[x + y*size]`` array (128 / 0) once all cells reported.

The cell actors and their 18 messages per cell per generation are replaced by one ``Board`` (HBM,
HIP kernels).  ``update_view()`` keeps the reference's observable contract: it posts
``UpdateView.Reset`` and then one ``Update(alive, {x; y})`` per cell in ``applyGrid`` order -- or, with
``emit="pixels"``, hands the agent the frame rendered on the GPU (``gol_render_gray8``).
"""
from __future__ import annotations

import os
import threading
import time
from typing import Callable, Optional

import numpy as np

from .board import INIT_DOTNET_MOD2, TORUS, Board
from .logic import Grid, Location, UpdateView, grid


class UpdateAgent:
    """GameOfLifeUI.fs:13-35: Reset starts a new dictionary; each Update inserts; when the dictionary
    holds every cell the pixels are filled and ``on_frame(pixels)`` is called (the WPF WritePixels)."""

    def __init__(self, g: Grid = grid, alive_value: int = 128, on_frame: Optional[Callable[[np.ndarray], None]] = None):
        self.grid = g
        self.alive_value = alive_value
        self.pixels = np.zeros(g.Width * g.Height, dtype=np.uint8)
        self.on_frame = on_frame
        self.frames = 0
        self._states: dict = {}

    def post(self, msg: UpdateView) -> None:
        if msg.kind == "Reset":
            self._states = {}
            return
        self._states[msg.location] = msg.alive
        if len(self._states) == self.grid.Width * self.grid.Height:
            w = self.grid.Width
            for (x, y), alive in self._states.items():
                self.pixels[x + y * w] = self.alive_value if alive else 0
            self._frame()

    def post_frame(self, pixels: np.ndarray) -> None:
        """Fast path: a whole frame rendered on the GPU replaces W*H Update messages."""
        self.pixels = pixels
        self._frame()

    def _frame(self) -> None:
        self.frames += 1
        if self.on_frame is not None:
            self.on_frame(self.pixels)


class GameOfLife:
    """The object ``run()`` returns: owns the board, the agent and the optional timer (IDisposable)."""

    def __init__(self, board: Board, agent: UpdateAgent, emit: str):
        if emit not in ("updates", "pixels"):
            raise ValueError("emit must be 'updates' or 'pixels'")
        self.board, self.agent, self.emit = board, agent, emit
        self._timer: Optional[threading.Thread] = None
        self._stop = threading.Event()
        self._lock = threading.Lock()  # the reference's timer may re-enter updateView; serialise ticks

    def update_view(self) -> None:
        """GameOfLifeDriver.fs:32-34: one tick = UpdateView.Reset, then one generation for every cell."""
        with self._lock:
            self.agent.post(UpdateView.Reset())
            self.board.step(1)
            if self.emit == "pixels":
                self.agent.post_frame(self.board.render_gray8(self.agent.alive_value))
                return
            cells = self.board.get_cells()
            g = self.agent.grid
            for x in range(g.Width):  # applyGrid order, GameOfLifeLogic.fs:13-15
                col = cells[:, x]
                for y in range(g.Height):
                    self.agent.post(UpdateView.Update(bool(col[y]), Location(x, y)))

    def start(self, period_s: float) -> "GameOfLife":
        """GameOfLifeDriver.fs:38-40: a timer calling update_view every period."""

        def loop():
            while not self._stop.wait(period_s):
                self.update_view()

        self._timer = threading.Thread(target=loop, daemon=True)
        self._timer.start()
        return self

    def dispose(self) -> None:
        self._stop.set()
        if self._timer is not None:
            self._timer.join()
        self.board.close()

    def __enter__(self) -> "GameOfLife":
        return self

    def __exit__(self, *exc) -> None:
        self.dispose()


def run(
    g: Grid = grid,
    seed: Optional[int] = None,
    agent: Optional[UpdateAgent] = None,
    boundary: int = TORUS,
    period_s: Optional[float] = None,
    emit: str = "updates",
    tblock_k: int = 0,
    num_gpus: int = 1,
) -> GameOfLife:
    """GameOfLifeDriver.fs:13-41.  ``seed`` replaces ``int DateTime.Now.Ticks`` (L10) so runs are
    reproducible; the board is seeded x outer / y inner with ``Random.Next() % 2 = 0`` (L9-11,16-19).
    With ``period_s`` a timer ticks like L38-40 (reference: ProcessorCount * 70 ms).  ``num_gpus`` > 1
    spreads the board over that many GPUs of this process (row strips; needs a width divisible by 32)."""
    if seed is None:
        seed = int(time.time_ns() // 100) & 0xFFFFFFFF  # .NET ticks are 100 ns; `int` truncates to 32 bits
        seed = seed - (1 << 32) if seed >= (1 << 31) else seed
    board = Board(g.Width, g.Height, boundary, tblock_k, num_gpus=num_gpus)
    board.seed_dotnet(seed, INIT_DOTNET_MOD2)
    game = GameOfLife(board, agent or UpdateAgent(g), emit)
    if period_s is not None:
        game.start(period_s)
    return game


def default_period_s() -> float:
    """GameOfLifeDriver.fs:38: Environment.ProcessorCount * 70 ms."""
    return (os.cpu_count() or 1) * 0.070
