"""MNIST fully connected (BASELINE config 1): 784 -> all2all_tanh(100) ->
softmax(10).  ``python -m veles_amd samples/mnist_fc.py -`` (CPU: -a cpu)."""
from veles_amd.models import StandardWorkflow
from veles_amd.utils.config import root, fix_contents
import veles_amd.loader  # noqa: F401


def run(load, main):
    cfg = fix_contents(root.mnist_fc)
    load(StandardWorkflow, loader_name=cfg["loader_name"],
         loader_config=cfg["loader"], layers=cfg["layers"],
         decision_config=cfg["decision"],
         snapshotter_config=cfg.get("snapshotter"))
    main()
