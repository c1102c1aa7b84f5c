"""bayesdll.csghmc_fs is bayesdll_amd.csghmc_fs (see bayesdll/__init__.py)."""
import sys

from bayesdll_amd import csghmc_fs as _impl

sys.modules[__name__] = _impl
