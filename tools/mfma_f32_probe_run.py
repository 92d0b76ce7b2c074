"""Runs tools/mfma_f32_probe (built from tools/mfma_f32_probe.hip in the build container) as a
child process and prints its report (gpu.sh py= step)."""
import os
import subprocess
import sys

exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mfma_f32_probe")
sys.exit(subprocess.run([exe]).returncode)
