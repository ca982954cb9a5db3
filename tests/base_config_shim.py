"""Parameter sets used by the golden generator, as plain dicts (no reference import)."""


def layer_weights(L):
    if L == 1:
        return [1.0]
    return [1.0 - 0.5 * (i / (L - 1)) for i in range(L)]


def coverage_config(L):
    return dict(alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25, layer_weights=layer_weights(L),
                bits=(2, 4, 8), ratios=(0.8, 0.6, 0.4))
