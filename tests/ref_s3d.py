"""Independent NCDHW functional evaluation of an S3D-G state_dict (test oracle).

Written directly from the reference's documented semantics: conv(bias=False)
-> BatchNorm3d -> ReLU units, full-channel (2+1)D "separable" convs, SelfGating, TF-SAME
zero-padded ceil-mode max pools, -inf padded 3x3x3 stride-1 branch pool, mean pool, fc.
It reads parameters by their state_dict names, so it checks key naming as well as math.
"""
import torch
import torch.nn.functional as F

BLOCKS = [("mixed_3b", False), ("mixed_3c", False), ("maxpool_4a", True), ("mixed_4b", False),
          ("mixed_4c", False), ("mixed_4d", False), ("mixed_4e", False), ("mixed_4f", False),
          ("maxpool_5a", True), ("mixed_5b", False), ("mixed_5c", False)]
POOLS = {"maxpool_2a": ((1, 3, 3), (1, 2, 2)), "maxpool_3a": ((1, 3, 3), (1, 2, 2)),
         "maxpool_4a": ((3, 3, 3), (2, 2, 2)), "maxpool_5a": ((2, 2, 2), (2, 2, 2))}


def _bn(x, sd, p, training):
    return F.batch_norm(x, sd[p + ".running_mean"].clone(), sd[p + ".running_var"].clone(), sd[p + ".weight"],
                        sd[p + ".bias"], training, 0.1, 1e-5)


def unit(x, sd, p, stride=1, padding=0, training=True):
    w = sd[p + ".conv1.weight"]
    if (p + ".conv2.weight") in sd:  # separable: [1,k,k] then [k,1,1]
        x = F.relu(_bn(F.conv3d(x, w, None, (1, stride, stride), (0, padding, padding)), sd, p + ".bn1", training))
        w2 = sd[p + ".conv2.weight"]
        return F.relu(_bn(F.conv3d(x, w2, None, (stride, 1, 1), (padding, 0, 0)), sd, p + ".bn2", training))
    return F.relu(_bn(F.conv3d(x, w, None, stride, padding), sd, p + ".bn1", training))


def gate(x, sd, p):
    g = torch.sigmoid(F.linear(x.mean(dim=(2, 3, 4)), sd[p + ".fc.weight"], sd[p + ".fc.bias"]))
    return x * g[:, :, None, None, None]


def tf_pool(x, k, s):
    pads = []
    for kk, ss in zip(reversed(k), reversed(s)):
        a = max(kk - ss, 0)
        pads += [a // 2, a - a // 2]
    return F.max_pool3d(F.pad(x, pads, value=0.0), k, s, ceil_mode=True)


def inception(x, sd, p, training):
    b0 = unit(x, sd, p + ".conv_b0", training=training)
    b1 = unit(unit(x, sd, p + ".conv_b1_a", training=training), sd, p + ".conv_b1_b", 1, 1, training)
    b2 = unit(unit(x, sd, p + ".conv_b2_a", training=training), sd, p + ".conv_b2_b", 1, 1, training)
    b3 = unit(F.max_pool3d(x, 3, 1, 1), sd, p + ".conv_b3_b", training=training)
    outs = [gate(b, sd, f"{p}.gating_b{i}") for i, b in enumerate((b0, b1, b2, b3))]
    return torch.cat(outs, dim=1)


def space_to_depth(x):
    """[B, C, T, H, W] -> [B, 8C, T/2, H/2, W/2], channel = ((dt*2 + dh)*2 + dw)*C + c
    (the public S3D_HowTo100M weights' input transform)."""
    b, c, t, h, w = x.shape
    x = x.reshape(b, c, t // 2, 2, h // 2, 2, w // 2, 2)
    out = torch.empty(b, 8 * c, t // 2, h // 2, w // 2, dtype=x.dtype)
    for dt in range(2):
        for dh in range(2):
            for dw in range(2):
                j = (dt * 2 + dh) * 2 + dw
                out[:, j * c:(j + 1) * c] = x[:, :, :, dt, :, dh, :, dw]
    return out


def s3d_video(sd, video_ncdhw, training=True, mixed5c=False):
    w = sd["conv1.conv1.weight"]
    if w.shape[1] == 24:  # space-to-depth stem: [2,4,4] conv, pad (1,2,2), BN+ReLU, then crop 1 in T/H/W
        x = F.relu(_bn(F.conv3d(space_to_depth(video_ncdhw), w, None, 1, (1, 2, 2)), sd, "conv1.bn1", training))
        x = x[:, :, 1:, 1:, 1:]
    else:
        x = F.relu(_bn(F.conv3d(video_ncdhw, w, None, 2, (1, 3, 3)), sd, "conv1.bn1", training))
    x = tf_pool(x, *POOLS["maxpool_2a"])
    x = unit(x, sd, "conv_2b", training=training)
    x = unit(x, sd, "conv_2c", 1, 1, training)
    x = gate(x, sd, "gating")
    x = tf_pool(x, *POOLS["maxpool_3a"])
    for name, is_pool in BLOCKS:
        if is_pool:
            x = tf_pool(x, *POOLS[name])
        elif name + ".conv_b0.conv1.weight" in sd:
            x = inception(x, sd, name, training)
    x = x.mean(dim=(2, 3, 4))
    if mixed5c:
        return x
    return F.linear(x, sd["fc.weight"], sd["fc.bias"])


def s3d_text(sd, tokens):
    e = F.embedding(tokens, sd["text_module.word_embd.weight"])
    h = F.relu(F.linear(e, sd["text_module.fc1.weight"], sd["text_module.fc1.bias"]))
    return F.linear(h.max(dim=1)[0], sd["text_module.fc2.weight"], sd["text_module.fc2.bias"])
