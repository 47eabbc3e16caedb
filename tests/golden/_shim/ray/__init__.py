"""Stand-in for ray, used ONLY by tests/golden/make_golden.py to import the read-only
reference's introgression model build (int_get_tab.py:5, get_tab.py:5) in this container,
where ray is not installed.  Not reference code; never ships."""
from . import util  # noqa: F401
