"""Mirror of the reference's F# grid/generation types (``GameOfLife/GameOfLife/GameOfLifeLogic.fs``).

Only the types the drop-in keeps are restated; the per-cell ``CellMessage`` protocol (L17-22) and
``createCell`` (L39-71) are what the HIP engine replaces (see ``board.Board``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, NamedTuple, Optional

size = 100  # GameOfLifeLogic.fs:5 (also GameofLife.fs:18)


class Grid(NamedTuple):  # GameOfLifeLogic.fs:6
    Width: int
    Height: int


grid = Grid(size, size)  # GameOfLifeLogic.fs:8
gridProduct = size * size  # GameOfLifeLogic.fs:7


class Location(NamedTuple):  # GameOfLifeLogic.fs:10-11 ([<Struct>] {x; y})
    x: int
    y: int


def apply_grid(f: Callable[[int, int], None], g: Grid = grid) -> None:
    """GameOfLifeLogic.fs:13-15: x outer, y inner."""
    for x in range(g.Width):
        for y in range(g.Height):
            f(x, y)


@dataclass(frozen=True)
class UpdateView:
    """GameOfLifeLogic.fs:32-35: ``Reset | Update of bool * Location``."""

    kind: str  # "Reset" | "Update"
    alive: bool = False
    location: Optional[Location] = None

    @staticmethod
    def Reset() -> "UpdateView":
        return UpdateView("Reset")

    @staticmethod
    def Update(alive: bool, location: Location) -> "UpdateView":
        return UpdateView("Update", bool(alive), location)
