"""``python -m pfml ...`` entry point (see pfml.cli)."""
import sys

from .cli import main

sys.exit(main())
