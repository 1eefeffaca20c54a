"""bench.py's stdout carries exactly ONE JSON line: anything else written to
fd 1 by native code (RCCL prints a version banner to C stdout when a
communicator comes up -- seen on the GPU box at world 1) goes to stderr."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_only_the_json_line_reaches_stdout():
    code = ("import os, sys, ctypes; sys.path.insert(0, %r); import bench\n"
            "fd = bench._stdout_for_json_only()\n"
            "print('python noise')\n"
            "libc = ctypes.CDLL(None); libc.puts(b'RCCL version : banner'); libc.fflush(None)\n"
            "os.write(1, b'raw fd noise\\n')\n"
            "bench.emit(fd, {'metric': 'm', 'value': 1.5})\n") % ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert len(lines) == 1 and json.loads(lines[0]) == {"metric": "m", "value": 1.5}, r.stdout
    assert "RCCL version" in r.stderr and "python noise" in r.stderr and "raw fd noise" in r.stderr
