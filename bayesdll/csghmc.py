"""bayesdll.csghmc is bayesdll_amd.csghmc (see bayesdll/__init__.py)."""
import sys

from bayesdll_amd import csghmc as _impl

sys.modules[__name__] = _impl
