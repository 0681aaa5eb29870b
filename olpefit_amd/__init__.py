"""olpefit_amd -- MI355X-native implementation of the apf_step2 Gibbs/MH hot path of
logan-pearce/olpefit (LAPF): per-proposal evaluation of the 2-Gaussian x N-source PSF
model and its chi^2 residual, for many independent walkers, as hand-written HIP for
gfx950 behind a C-ABI (include/olpe.h, libolpe.so)."""
__version__ = "0.1.0"
