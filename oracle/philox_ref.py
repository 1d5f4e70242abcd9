"""TEST INFRASTRUCTURE ONLY — CPU oracle.  Never imported by the product path.

Philox4x32-10 counter-based RNG (Salmon et al., SC'11, "Parallel random
numbers: as easy as 1, 2, 3"; constants and round schedule of Random123's
philox4x32_R with R = 10), restated in pure Python integers.  This is the
stream the build uses for spawn proposals (the reference draws them from the
Simulator's np_random in gym-duckietown's reset(); its exact stream cannot be
reproduced without the un-vendored package, so reset parity is defined
against this build-defined stream — see DESIGN.md "Reset").

Pinned by the Random123 known-answer vectors in tests/test_oracle_philox.py.
"""

M0 = 0xD2511F53
M1 = 0xCD9E8D57
W0 = 0x9E3779B9
W1 = 0xBB67AE85
MASK = 0xFFFFFFFF

# stream tags (4th counter word) — must match aido1_amd/csrc/dtsim.hip
TAG_TILE = 0x54494C45     # 'TILE': drivable-tile pick of one reset
TAG_SPAWN_A = 0x53504E41  # 'SPNA': proposal k -> (u_x, u_z)
TAG_SPAWN_B = 0x53504E42  # 'SPNB': proposal k -> u_angle


def philox4x32_10(ctr, key):
    c0, c1, c2, c3 = (int(v) & MASK for v in ctr)
    k0, k1 = (int(v) & MASK for v in key)
    for r in range(10):
        if r:
            k0 = (k0 + W0) & MASK
            k1 = (k1 + W1) & MASK
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> 32, p0 & MASK
        hi1, lo1 = p1 >> 32, p1 & MASK
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0), lo1, (hi0 ^ c3 ^ k1), lo0
    return c0, c1, c2, c3


def u01(a, b):
    """Two u32 words -> double in [0, 1) with 53 random bits."""
    return ((((a & MASK) << 32) | (b & MASK)) >> 11) * (1.0 / 9007199254740992.0)


def key_of(seed):
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    return seed & MASK, seed >> 32


def tile_uniform(seed, env_id, episode):
    w = philox4x32_10((0, episode, env_id, TAG_TILE), key_of(seed))
    return u01(w[0], w[1])


def spawn_uniforms(seed, env_id, episode, k):
    key = key_of(seed)
    a = philox4x32_10((k, episode, env_id, TAG_SPAWN_A), key)
    b = philox4x32_10((k, episode, env_id, TAG_SPAWN_B), key)
    return u01(a[0], a[1]), u01(a[2], a[3]), u01(b[0], b[1])
