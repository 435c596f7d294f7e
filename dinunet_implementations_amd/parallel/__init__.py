"""Sites as ranks: process group, aggregation engines, low-rank numerics."""
from .group import SiteGroup, current, init_sites, shutdown
from .engines import DSGDEngine, Engine, PowerSGDEngine, RankDADEngine, ENGINES, make_engine

__all__ = ["SiteGroup", "current", "init_sites", "shutdown", "Engine", "DSGDEngine",
           "RankDADEngine", "PowerSGDEngine", "ENGINES", "make_engine"]
