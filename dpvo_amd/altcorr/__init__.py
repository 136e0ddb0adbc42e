"""altcorr on MI355X: patch correlation (A-CORR) and patch extraction (A-PATCH).

Same entry points as dpvo/altcorr/correlation.py of cuteboyqq/DPVO
(`corr`, `patchify`, `CorrLayer`, `PatchLayer`), backed by the `cuda_corr`
HIP extension.  Extra: `corr_levels`, the fused all-levels call of
DPVO.corr (dpvo/dpvo.py:456-465) in one launch, and `to_channels_last`
(pyramids stored channels-last take the matrix-core correlation path), and
`insert_frame`, the one-launch channels-last frame insertion of all levels
(`insert_frame_ring`: ring slot read on the device, for graph replay).
"""
from .correlation import (  # noqa: F401
    BORDER_MODE,
    CorrLayer,
    PatchLayer,
    corr,
    corr_levels,
    insert_frame,
    insert_frame_ring,
    patchify,
    to_channels_last,
)
