"""Run a script against another build of the library (A/B tooling only).

Usage: python tools/with_lib.py <path/to/lib.so> <script.py> [args...]
Rebinds dialog_amd._lib.LIB_PATH before the script imports the package; the shipped binding
itself always loads the in-tree dialog_amd/libdialog_amd.so.
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from dialog_amd import _lib  # noqa: E402

if __name__ == "__main__":
    _lib.LIB_PATH = os.path.abspath(sys.argv[1])
    script = sys.argv[2]
    sys.argv = [script] + sys.argv[3:]
    sys.path.insert(0, os.path.dirname(os.path.abspath(script)))
    runpy.run_path(script, run_name="__main__")
