from . import reference
from ._ext import available as ext_available, ext
