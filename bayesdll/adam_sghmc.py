"""bayesdll.adam_sghmc is bayesdll_amd.adam_sghmc (see bayesdll/__init__.py)."""
import sys

from bayesdll_amd import adam_sghmc as _impl

sys.modules[__name__] = _impl
