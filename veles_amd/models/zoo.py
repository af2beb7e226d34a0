"""Benchmark topologies (BASELINE.json configs).  The reference
sample workflows lived in the absent Znicz submodule, so these are the
conventional definitions, written as StandardWorkflow ``layers`` lists.

* mnist_fc   : 784 -> all2all_tanh(100) -> softmax(10)   (export fixture)
* lenet      : Caffe LeNet (conv 20x5x5, pool, conv 50x5x5, pool, 500, 10)
* cifar_quick: Caffe cifar10_quick (3x conv 5x5 32/32/64 + pools, 64, 10)
* alexnet    : Caffe bvlc_alexnet, 227x227x3, grouped conv2/4/5, LRN
* vgg16      : VGG-16 (13 conv 3x3 + 5 pools, 4096-4096-1000)
"""
from __future__ import annotations

__all__ = ["mnist_fc", "lenet", "cifar_quick", "alexnet", "vgg16", "MODELS",
           "gd_params"]


def gd_params(lr=0.01, moment=0.9, decay=5e-4, lr_bias=None):
    return {"learning_rate": lr, "learning_rate_bias": lr_bias or 2 * lr,
            "gradient_moment": moment, "gradient_moment_bias": moment,
            "weights_decay": decay, "weights_decay_bias": 0.0}


def mnist_fc(lr=0.1):
    g = gd_params(lr, 0.9, 0.0, lr)
    return [{"type": "all2all_tanh", "->": {"output_sample_shape": 100},
             "<-": g},
            {"type": "softmax", "->": {"output_sample_shape": 10}, "<-": g}]


def lenet(lr=0.01):
    g = gd_params(lr, 0.9, 5e-4)
    return [
        {"type": "conv", "->": {"n_kernels": 20, "kx": 5, "ky": 5}, "<-": g},
        {"type": "max_pooling", "->": {"kx": 2, "ky": 2, "sliding": 2}},
        {"type": "conv", "->": {"n_kernels": 50, "kx": 5, "ky": 5}, "<-": g},
        {"type": "max_pooling", "->": {"kx": 2, "ky": 2, "sliding": 2}},
        {"type": "all2all_str", "->": {"output_sample_shape": 500}, "<-": g},
        {"type": "softmax", "->": {"output_sample_shape": 10}, "<-": g}]


def cifar_quick(lr=0.001):
    g = gd_params(lr, 0.9, 4e-3)
    pool = {"kx": 3, "ky": 3, "sliding": 2}
    return [
        {"type": "conv", "->": {"n_kernels": 32, "kx": 5, "ky": 5,
                                "padding": 2, "weights_stddev": 1e-4},
         "<-": g},
        {"type": "max_pooling", "->": dict(pool)},
        {"type": "activation_str"},
        {"type": "conv_str", "->": {"n_kernels": 32, "kx": 5, "ky": 5,
                                    "padding": 2, "weights_stddev": 0.01},
         "<-": g},
        {"type": "avg_pooling", "->": dict(pool)},
        {"type": "conv_str", "->": {"n_kernels": 64, "kx": 5, "ky": 5,
                                    "padding": 2, "weights_stddev": 0.01},
         "<-": g},
        {"type": "avg_pooling", "->": dict(pool)},
        {"type": "all2all", "->": {"output_sample_shape": 64,
                                   "weights_stddev": 0.1}, "<-": g},
        {"type": "softmax", "->": {"output_sample_shape": 10,
                                   "weights_stddev": 0.1}, "<-": g}]


def alexnet(lr=0.01, n_classes=1000):
    g = gd_params(lr, 0.9, 5e-4)
    lrn = {"n": 5, "alpha": 1e-4 / 5, "beta": 0.75, "k": 1.0}
    pool = {"kx": 3, "ky": 3, "sliding": 2}
    gw = dict(g)
    return [
        {"type": "conv_str", "name": "conv1",
         "->": {"n_kernels": 96, "kx": 11, "ky": 11, "sliding": 4,
                "weights_filling": "gaussian", "weights_stddev": 0.01,
                "bias_filling": "constant", "bias_stddev": 0.0}, "<-": gw},
        {"type": "norm", "name": "norm1", "->": dict(lrn)},
        {"type": "max_pooling", "name": "pool1", "->": dict(pool)},
        {"type": "conv_str", "name": "conv2",
         "->": {"n_kernels": 256, "kx": 5, "ky": 5, "padding": 2,
                "grouping": 2, "weights_filling": "gaussian",
                "weights_stddev": 0.01, "bias_filling": "constant",
                "bias_stddev": 0.1}, "<-": gw},
        {"type": "norm", "name": "norm2", "->": dict(lrn)},
        {"type": "max_pooling", "name": "pool2", "->": dict(pool)},
        {"type": "conv_str", "name": "conv3",
         "->": {"n_kernels": 384, "kx": 3, "ky": 3, "padding": 1,
                "weights_filling": "gaussian", "weights_stddev": 0.01,
                "bias_filling": "constant", "bias_stddev": 0.0}, "<-": gw},
        {"type": "conv_str", "name": "conv4",
         "->": {"n_kernels": 384, "kx": 3, "ky": 3, "padding": 1,
                "grouping": 2, "weights_filling": "gaussian",
                "weights_stddev": 0.01, "bias_filling": "constant",
                "bias_stddev": 0.1}, "<-": gw},
        {"type": "conv_str", "name": "conv5",
         "->": {"n_kernels": 256, "kx": 3, "ky": 3, "padding": 1,
                "grouping": 2, "weights_filling": "gaussian",
                "weights_stddev": 0.01, "bias_filling": "constant",
                "bias_stddev": 0.1}, "<-": gw},
        {"type": "max_pooling", "name": "pool5", "->": dict(pool)},
        {"type": "all2all_str", "name": "fc6",
         "->": {"output_sample_shape": 4096, "weights_filling": "gaussian",
                "weights_stddev": 0.005, "bias_filling": "constant",
                "bias_stddev": 0.1}, "<-": gw},
        {"type": "dropout", "name": "drop6", "->": {"dropout_ratio": 0.5}},
        {"type": "all2all_str", "name": "fc7",
         "->": {"output_sample_shape": 4096, "weights_filling": "gaussian",
                "weights_stddev": 0.005, "bias_filling": "constant",
                "bias_stddev": 0.1}, "<-": gw},
        {"type": "dropout", "name": "drop7", "->": {"dropout_ratio": 0.5}},
        {"type": "softmax", "name": "fc8",
         "->": {"output_sample_shape": n_classes,
                "weights_filling": "gaussian", "weights_stddev": 0.01,
                "bias_filling": "constant", "bias_stddev": 0.0}, "<-": gw}]


def vgg16(lr=0.01, n_classes=1000):
    g = gd_params(lr, 0.9, 5e-4)
    layers = []
    cfg = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512,
           "M", 512, 512, 512, "M"]
    ci = 0
    for c in cfg:
        if c == "M":
            layers.append({"type": "max_pooling",
                           "->": {"kx": 2, "ky": 2, "sliding": 2}})
        else:
            ci += 1
            layers.append({"type": "conv_str", "name": "conv%d" % ci,
                           "->": {"n_kernels": c, "kx": 3, "ky": 3,
                                  "padding": 1, "weights_filling": "gaussian",
                                  "weights_stddev": 0.01,
                                  "bias_filling": "constant",
                                  "bias_stddev": 0.0}, "<-": dict(g)})
    for i, n in enumerate((4096, 4096)):
        layers.append({"type": "all2all_str", "name": "fc%d" % (6 + i),
                       "->": {"output_sample_shape": n,
                              "weights_filling": "gaussian",
                              "weights_stddev": 0.005}, "<-": dict(g)})
        layers.append({"type": "dropout", "->": {"dropout_ratio": 0.5}})
    layers.append({"type": "softmax", "name": "fc8",
                   "->": {"output_sample_shape": n_classes,
                          "weights_filling": "gaussian",
                          "weights_stddev": 0.01}, "<-": dict(g)})
    return layers


MODELS = {
    "mnist_fc": (mnist_fc, "mnist"),
    "lenet": (lenet, "mnist"),
    "cifar_quick": (cifar_quick, "cifar10"),
    "alexnet": (alexnet, "imagenet"),
    "vgg16": (vgg16, "imagenet224"),
}
