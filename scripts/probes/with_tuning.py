#!/usr/bin/env python3
"""Run a script with knobs.TUNING overrides: with_tuning.py NAME=VALUE ... -- script.py args"""
import ast
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from hipsnapshot import knobs  # noqa: E402

i = sys.argv.index("--")
for kv in sys.argv[1:i]:
    k, v = kv.split("=", 1)
    setattr(knobs.TUNING, k, ast.literal_eval(v))
sys.argv = sys.argv[i + 1:]
sys.path.insert(0, os.path.dirname(os.path.abspath(sys.argv[0])))
runpy.run_path(sys.argv[0], run_name="__main__")
