from .spec import Conv, Dense, LRN, MaxPool, ModelSpec  # noqa: F401
from .registry import MODELS, get_model, lenet5, mlp, reference_cnn  # noqa: F401
