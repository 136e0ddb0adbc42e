"""A/B of the stale-granule condition (tests/test_granule_stale_gpu.py) on two
builds: process A runs one BA call and saves its workspace, fresh process B
loads those bytes into its own workspace and runs its first BA call on other
measurements.  Prints B's outcome for each tree given on the command line
(e.g. the round-4 build and this one).

    python scripts/stale_granule_demo.py <tree> [<tree> ...]
"""
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))

from test_granule_stale_gpu import CHILD  # noqa: E402


def main():
    for tree in sys.argv[1:]:
        tree = os.path.abspath(tree)
        with tempfile.TemporaryDirectory() as d:
            path = os.path.join(d, "ws.npy")
            env = dict(os.environ, PYTHONPATH=os.path.join(tree, "tests"))
            res = []
            for role in ("A", "B"):
                r = subprocess.run([sys.executable, "-c", CHILD, tree, role, path], env=env,
                                   capture_output=True, text=True, timeout=180)
                res.append((role, r.returncode, (r.stdout + r.stderr).strip().splitlines()[-1:]))
                if r.returncode:
                    break
            print(tree, res, flush=True)


if __name__ == "__main__":
    main()
