"""bayesdll.sgld is bayesdll_amd.sgld (see bayesdll/__init__.py)."""
import sys

from bayesdll_amd import sgld as _impl

sys.modules[__name__] = _impl
