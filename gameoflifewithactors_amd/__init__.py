"""gameoflifewithactors_amd -- MI355X (gfx950) Game of Life engine.

Replaces the per-cell actor loop of rikace/GameOfLifeWithActors (F# MailboxProcessor / Akka.NET cells
applying B3/S23 every generation) with HIP kernels behind a C ABI (``include/gol/gol.h``,
``libgol_hip.so``).  Python pieces:

* ``board.Board``     -- one board in HBM; the C ABI's board handle
* ``logic``           -- Grid / Location / UpdateView / apply_grid (GameOfLifeLogic.fs)
* ``driver``          -- run() / update_view() / UpdateAgent (GameOfLifeDriver.fs, GameOfLifeUI.fs)
* ``strips``          -- multi-GPU row strips with the halo exchange (one process per GPU)
"""
from ._lib import BOUNDED, INIT_DOTNET_MOD2, INIT_DOTNET_NEXT2, TORUS, GolError  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):  # lazy: importing the package must not require the shared library
    if name in ("Board", "hash_finalize"):
        from . import board

        return getattr(board, name)
    raise AttributeError(name)
