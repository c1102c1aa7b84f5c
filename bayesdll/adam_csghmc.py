"""bayesdll.adam_csghmc is bayesdll_amd.adam_csghmc (see bayesdll/__init__.py)."""
import sys

from bayesdll_amd import adam_csghmc as _impl

sys.modules[__name__] = _impl
