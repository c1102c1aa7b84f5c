"""bayesdll.cyclical is bayesdll_amd.cyclical (see bayesdll/__init__.py)."""
import sys

from bayesdll_amd import cyclical as _impl

sys.modules[__name__] = _impl
