"""paddle.nn.functional (reference: python/paddle/nn/functional/__init__.py)."""
from .activation import *  # noqa: F401,F403
from .common import *  # noqa: F401,F403
from .conv import *  # noqa: F401,F403
from .loss import *  # noqa: F401,F403
from .norm import *  # noqa: F401,F403
from .attention import *  # noqa: F401,F403
from ..decode import gather_tree  # noqa: F401,E402
