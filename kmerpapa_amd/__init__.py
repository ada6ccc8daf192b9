"""kmerpapa_amd -- MI355X-native k-mer pattern partition (penalized-likelihood lattice DP).

Drop-in for the hot path of BesenbacherLab/kmerPaPa v0.2.4: same module names and
function signatures for the DP drivers, pattern algebra and CV tools; the lattice DP runs
in hand-written gfx950 HIP kernels behind a C-ABI (include/kmerpapa_hip.h).
"""
__all__ = []
__version__ = "0.2.4"
