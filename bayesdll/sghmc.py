"""bayesdll.sghmc is bayesdll_amd.sghmc (see bayesdll/__init__.py)."""
import sys

from bayesdll_amd import sghmc as _impl

sys.modules[__name__] = _impl
