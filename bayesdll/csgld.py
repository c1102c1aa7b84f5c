"""bayesdll.csgld is bayesdll_amd.csgld (see bayesdll/__init__.py)."""
import sys

from bayesdll_amd import csgld as _impl

sys.modules[__name__] = _impl
