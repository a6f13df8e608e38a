"""pygcransac: drop-in package of yuvalnis/graph-cut-ransac backed by the
MI355X engine (same layout as the reference's src/pygcransac/__init__.py:1)."""
from .pygcransac import *  # noqa: F401,F403
from .pygcransac import __all__  # noqa: F401
