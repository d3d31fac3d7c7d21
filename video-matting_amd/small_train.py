"""Reference-named entry point: `import small_train` (small_train.py:1-112): small_training's loop and
train(learning_rate) (vmatting.procedures) over the device SmallTrainer (vmatting.small_train)."""
from vmatting.procedures import small_train as train  # noqa: F401
from vmatting.procedures import small_training  # noqa: F401
from vmatting.small_train import SmallTrainer  # noqa: F401
