"""`python -m kmerpapa_amd` entry point (reference: src/kmerpapa/__main__.py)."""
import sys

from kmerpapa_amd.cli import main

if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
