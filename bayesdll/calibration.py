"""bayesdll.calibration is bayesdll_amd.calibration (see bayesdll/__init__.py)."""
import sys

from bayesdll_amd import calibration as _impl

sys.modules[__name__] = _impl
