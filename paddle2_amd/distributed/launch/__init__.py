from .main import launch  # noqa
