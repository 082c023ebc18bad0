from .common import *  # noqa: F401,F403
from .layers import Layer  # noqa: F401
from .transformer import *  # noqa: F401,F403
from .rnn import RNN, BiRNN, RNNCellBase, birnn, rnn  # noqa: F401
