"""basecount_amd — MI355X-native per-position pileup counter, drop-in for tombch/basecount.

``from basecount_amd import BaseCount`` mirrors ``from basecount import BaseCount``
(/root/reference/basecount/__init__.py:1); ``basecount_amd.count.bcount`` mirrors the reference's
native ``count.bcount`` (count.cpp:102-105).  The counting and statistics run on gfx950 HIP kernels
(``libbasecount_hip.so``); BAM decode and text output run on the host (``libbcio.so``).
"""
from .main import BaseCount  # noqa: F401
from .version import __version__  # noqa: F401
