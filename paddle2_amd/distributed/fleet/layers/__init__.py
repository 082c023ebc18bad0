from . import mpu  # noqa
