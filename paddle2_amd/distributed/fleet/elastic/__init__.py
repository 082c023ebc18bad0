"""Elastic training (reference: python/paddle/distributed/fleet/elastic/__init__.py, manager.py)."""
from .manager import (ELASTIC_AUTO_PARALLEL_EXIT_CODE, ELASTIC_EXIT_CODE, ELASTIC_TIMEOUT, ELASTIC_TTL,  # noqa
                      ElasticManager, ElasticStatus, LauncherInterface)


def enable_elastic(args, distribute_mode=None):
    n = str(getattr(args, "nnodes", "1"))
    return ":" in n or int(getattr(args, "elastic_level", -1)) >= 1


def launch_elastic(args, distribute_mode=None):
    from ...launch.main import launch

    return launch(args)
