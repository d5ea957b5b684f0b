"""One cooperative-pass launch on a mid-size board (profiling target): python tools/coop_one.py W H gens [boundary]"""
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from gameoflifewithactors_amd import Board  # noqa: E402

W, H, G = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
bnd = int(sys.argv[4]) if len(sys.argv) > 4 else 0
with Board(W, H, bnd) as b:
    b.seed_splitmix(7)
    b.step(G)
    b.step(G)
    b.synchronize()
