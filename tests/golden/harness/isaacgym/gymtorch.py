"""Stand-in for isaacgym.gymtorch: the FakeGym already hands out torch tensors."""


def wrap_tensor(t):
    return t


def unwrap_tensor(t):
    return t
