def to_2tuple(x):
    return x if isinstance(x, tuple) else (x, x)
