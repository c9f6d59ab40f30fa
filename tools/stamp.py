#!/usr/bin/env python3
"""Identity of a profiler record: which library and which sources produced it.

    python3 tools/stamp.py <out.json> <config> <command...>

Writes {config, lib_sha256, src_sha256, utc, host, command}: lib_sha256 of the liboceanhip.so that
ran, src_sha256 over the library's sources (csrc/*, include/ocean/ocean.h).  bench.py picks the
profiler record of a config whose stamp matches the library it loaded (then the sources, then the
newest stamp), never by directory name.  tools/pmc_summary.py adds the git HEAD."""
import datetime
import hashlib
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "ocean-simulation_amd", "ocean_hip", "liboceanhip.so")
SRC_DIRS = [os.path.join(ROOT, "ocean-simulation_amd", "csrc")]
SRC_FILES = [os.path.join(ROOT, "include", "ocean", "ocean.h")]


def file_sha(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def lib_sha(path=LIB):
    return file_sha(path) if os.path.exists(path) else None


def src_sha():
    h = hashlib.sha256()
    files = sorted(os.path.join(d, f) for d in SRC_DIRS for f in os.listdir(d)) + SRC_FILES
    for p in files:
        h.update(os.path.relpath(p, ROOT).encode())
        h.update(open(p, "rb").read())
    return h.hexdigest()


def stamp(config, command):
    return {"config": config, "lib_sha256": lib_sha(), "src_sha256": src_sha(),
            "utc": datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ"),
            "host": socket.gethostname(), "command": command}


CEILING_TOOLS = {"wrbench.txt": "wrbench.hip", "aqbench.txt": "aqbench.hip", "bqbench.txt": "bqbench.hip"}


def code_sha(path):
    """sha256 of a micro-benchmark's code: its lines with // comments and blank lines dropped, so an
    edit of a comment does not orphan the records the tool made."""
    h = hashlib.sha256()
    for line in open(path):
        code = line.split("//", 1)[0].rstrip()
        if code:
            h.update(code.encode() + b"\n")
    return h.hexdigest()


def ceiling_stamp(utc=None, git_head=None):
    """Identity of a directory of micro-benchmark records (wrbench / aqbench / bqbench .txt): the code
    sha256 of each tool and when it ran.  bench.py quotes the newest record made by the current code
    of the tool (then the newest at all), whatever the directory is called."""
    tools = os.path.join(ROOT, "tools")
    return {"kind": "ceilings",
            "utc": utc or datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ"),
            "host": socket.gethostname(), "git_head": git_head,
            "tool_code_sha256": {t: code_sha(os.path.join(tools, t)) for t in sorted(set(CEILING_TOOLS.values()))}}


if __name__ == "__main__":
    if sys.argv[1] == "--ceilings":  # stamp.py --ceilings <dir> [utc] [git_head]
        d = sys.argv[2]
        json.dump(ceiling_stamp(*(sys.argv[3:5])), open(os.path.join(d, "ceilings.json"), "w"), indent=1)
        sys.exit(0)
    out, config, cmd = sys.argv[1], sys.argv[2], " ".join(sys.argv[3:])
    json.dump(stamp(config, cmd), open(out, "w"), indent=1)
