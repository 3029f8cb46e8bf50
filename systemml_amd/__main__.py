import sys

from .api.cli import main

sys.exit(main())
