"""Engine servers (reference C28: jubatus/server/server/*_serv.cpp).

``SERVERS[engine]`` -> "module:Class" of the engine glue; ``get_serv`` imports
lazily so a server process only loads its own engine.
"""
from __future__ import annotations

import importlib

SERVERS = {
    "classifier": "classifier_serv:ClassifierServ",
    "regression": "regression_serv:RegressionServ",
    "recommender": "recommender_serv:RecommenderServ",
    "nearest_neighbor": "nearest_neighbor_serv:NearestNeighborServ",
    "anomaly": "anomaly_serv:AnomalyServ",
    "clustering": "clustering_serv:ClusteringServ",
    "graph": "graph_serv:GraphServ",
    "bandit": "bandit_serv:BanditServ",
    "burst": "burst_serv:BurstServ",
    "stat": "stat_serv:StatServ",
    "weight": "weight_serv:WeightServ",
}


def get_serv(engine: str):
    mod, cls = SERVERS[engine].split(":")
    return getattr(importlib.import_module(f"{__name__}.{mod}"), cls)
