import sys

from .pool import main

sys.exit(main())
