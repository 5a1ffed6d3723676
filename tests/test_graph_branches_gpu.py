"""A fork/join hipGraph: two independent chains of C-ABI launches captured as
branches of ONE graph (event record on the capturing stream, a side stream waits on it, each
stream enqueues its chain, the capturing stream joins the side stream before the capture ends)
instantiate, replay and give bitwise the outputs of the same chains captured serially
(tools/graph_branches.py; its timing -- the branches serialise on this stack -- is in
profiles/NOTES.md round 5).  Run in its own process: the probe owns its streams and graphs."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


def test_fork_join_graph_bitwise_equals_serial(cuda):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "graph_branches.py"), "8"],
                       capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "fork/join graph captured and instantiated" in r.stdout
    assert "outputs bitwise equal: True" in r.stdout
