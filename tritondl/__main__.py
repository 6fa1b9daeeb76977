"""``python -m tritondl`` — run the ingest worker (reference ``cmd/downloader``)."""

import sys

from .service import main

sys.exit(main())
