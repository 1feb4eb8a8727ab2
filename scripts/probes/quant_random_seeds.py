import os, sys, random, math, tempfile
sys.path[:0]=[os.getcwd(), os.path.join(os.getcwd(),'tests')]
import torch, test_quant_random as t
for seed in (101, 129, 220):
    try:
        t._round_trip(tempfile.mkdtemp(), seed, "cuda:0"); print(seed, "ok")
    except AssertionError as e:
        print(seed, "FAIL", str(e)[:200])
