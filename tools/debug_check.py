import sys, os, json
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_sudoku_solver_amd import SudokuEngine, synth
mode = sys.argv[1]
eng = SudokuEngine(0)
cases = json.load(open("tests/golden/check_cases.json"))["cases"]
boards = np.array([c["board"] for c in cases], dtype=np.uint8)
if mode == "a":
    print(eng.check_batch(boards[:1]))
elif mode == "b":
    print(eng.check_batch(boards)[:5]); print(eng.check_batch(boards[:1]))
elif mode == "c":
    for n in (1, 2, 3, 130, 131, 132):
        print(n, eng.check_batch(boards[:n])[:3], flush=True)
elif mode == "d":
    b = synth.parse(synth.WIKI_SOLUTION)[None]
    print(eng.check_batch(b))
