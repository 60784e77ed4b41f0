"""`python -m basecount_amd BAM [...]` — the reference's `basecount` console script (setup.py:16)."""
from .main import run

if __name__ == "__main__":
    run()
