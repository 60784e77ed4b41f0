"""`python -m basecount_amd BAM [...]` — the reference's `basecount` console script (setup.py:16)."""
import faulthandler
import os

from .main import run

if __name__ == "__main__":
    # diagnostic: BASECOUNT_HANG_DUMP=<seconds> prints every thread's stack to stderr once the
    # command has run that long (a multi-rank run waiting in a collective shows where)
    if os.environ.get("BASECOUNT_HANG_DUMP"):
        faulthandler.dump_traceback_later(float(os.environ["BASECOUNT_HANG_DUMP"]), exit=False)
    run()
