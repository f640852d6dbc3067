"""parprint (reference lib/Printing.py:4-6): print on rank 0 only."""
import os


def _rank():
    for k in ("RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK"):
        if k in os.environ:
            return int(os.environ[k])
    return 0


def parprint(*args, **kwargs):
    if _rank() == 0:
        print(*args, **kwargs)
