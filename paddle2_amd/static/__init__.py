"""paddle.static — placeholder replaced by the Program/Executor implementation (static/program.py)."""
from .program import *  # noqa: F401,F403
