"""ORACLE — test infrastructure only.

CPU restatements of the reference's hot path (akshatvasisht/janus) used as the
checker for the MI355X implementation in ``janus_amd``. Nothing in ``janus_amd/``
imports, links or executes anything under ``oracle/``; only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may.

Pinning status per sub-path is recorded in each module header and in DESIGN.md.
"""
import os

ORACLE_DIR = os.path.dirname(os.path.abspath(__file__))
BUILD_DIR = os.path.join(ORACLE_DIR, "_build")


def build() -> None:
    """Compile the oracle's C restatements (oracle/Makefile -> oracle/_build/)."""
    import subprocess
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
