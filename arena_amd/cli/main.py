"""`arena` entry point (reference: cmd/arena/main.go:12-39).

``--pprof`` is detected by scanning raw argv BEFORE parsing (so it works on every subcommand, as in
the reference) and writes a cProfile dump of the CLI itself to /tmp/cpu_profile.
"""
from __future__ import annotations

import os
import sys


def _pprof_enabled(argv) -> bool:
    return any(a == "--pprof" or a.startswith("--pprof=") and a.split("=", 1)[1] != "false"
               for a in argv)


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    from .commands import run
    if _pprof_enabled(argv):
        import cProfile
        path = os.environ.get("ARENA_PPROF_PATH", "/tmp/cpu_profile")
        prof = cProfile.Profile()
        prof.enable()
        try:
            rc = run(argv)
        finally:
            prof.disable()
            prof.dump_stats(path)
        return rc
    return run(argv)


if __name__ == "__main__":
    sys.exit(main())
