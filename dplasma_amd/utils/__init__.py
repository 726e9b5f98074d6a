from . import flops, lcg  # noqa: F401
from .info import Info, info_create  # noqa: F401
