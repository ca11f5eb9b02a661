"""torchOptics-compatible shim backed by libhbx.so.

The reference imports ``torchOptics.optics as tt`` and
``torchOptics.metrics as tm``; with this package's parent directory on
sys.path those imports resolve here and the hot operator (tt.simulate) runs
as HIP on the MI355X."""
from . import metrics, optics  # noqa: F401
