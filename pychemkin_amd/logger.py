"""Package logger (name-compatible with the reference's ``ck.logger``, logger.py:44-127).

The reference forces DEBUG to stderr at import (logger.py:125-127); this package defaults to
WARNING.
"""
import logging

logger = logging.getLogger("pychemkin_amd")
if not logger.handlers:
    _h = logging.StreamHandler()
    _h.setFormatter(logging.Formatter("%(levelname)s: %(message)s"))
    logger.addHandler(_h)
logger.setLevel(logging.WARNING)
