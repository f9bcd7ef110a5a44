"""``python -m singa_amd`` == the reference ``singa`` binary (src/main.cc)."""
import sys

from .main import main

sys.exit(main())
