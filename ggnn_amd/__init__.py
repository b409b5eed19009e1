"""ggnn_amd -- MI355X-native GGNN propagation engine (drop-in for the hot path
of crismolav/ggnn's DenseGGNNChemModel.compute_final_node_representations)."""
from .engine import PropagationEngine, WeightPack  # noqa: F401

__version__ = "0.1.0"
