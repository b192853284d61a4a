"""``python -m gol_amd <pattern> <worldSize> <iterations> <threadsPerBlock> <output_on_off>``

Same contract as the reference binary (gol-main.c:43-53) via the native CLI driver.
"""
import sys

from ._native import _gol

if __name__ == "__main__":
    sys.exit(_gol.run_cli(["gol", *sys.argv[1:]]))
