# The drop-in provides miscc.config and miscc.DAMSM_losses; the reference's
# other miscc modules (miscc/utils.py: image saving, train.py:22) keep coming
# from the reference tree when it follows this package on sys.path.
from pkgutil import extend_path

__path__ = extend_path(__path__, __name__)
