__version__ = "1.7.2"  # the reference's version string (basecount/version.py:1), printed by -v
