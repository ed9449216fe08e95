"""Same-named replacement for the reference's psf_fft module (psf_fft.py), backed by rocFFT.

Put akbraytracing_amd/dropin first on sys.path and `from psf_fft import compute_psf_fft,
psf_to_db` (AKB_raytrace_20250312.py:12, psf_fft_example.py:5) resolves here unmodified.
"""
from akbraytracing_amd.psf import compute_psf_fft, ensure_even_size, psf_to_db

__all__ = ["compute_psf_fft", "psf_to_db", "ensure_even_size"]
