"""MI355X-native (gfx950) training path for the mr_gen listener head-motion models.

Importing the package is cheap and GPU-free; the HIP library (``libmrg.so``)
is loaded on first use by ``multimodalreactiongeneration_amd._lib``.
"""
__version__ = "0.1.0"
