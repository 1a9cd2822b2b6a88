"""Training / evaluation engine: device-resident loops, HIP-graph step, arena Adam."""
from .evaluate import evaluate_model  # noqa: F401
from .graph import GraphedTrainStep  # noqa: F401
from .infer import GraphedForward, predict  # noqa: F401
from .optim import ArenaAdam  # noqa: F401
from .train import make_kd_step_fn, make_step_fn, train_model  # noqa: F401
