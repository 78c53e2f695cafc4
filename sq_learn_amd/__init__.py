"""sq_learn_amd - an MI355X-native (gfx950) quantum-simulated machine learning
framework with the capabilities of federicomegler/sq-learn."""
__version__ = "0.1.0"
