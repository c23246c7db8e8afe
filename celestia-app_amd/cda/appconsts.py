"""Constants mirrored from pkg/appconsts (celestia-app @ 2025-02-13)."""
SHARE_SIZE = 512                 # global_consts.go:29
NAMESPACE_VERSION_SIZE = 1
NAMESPACE_ID_SIZE = 28
NAMESPACE_SIZE = 29              # global_consts.go:26
MIN_SQUARE_SIZE = 1              # global_consts.go MinSquareSize
MIN_SHARE_COUNT = 1
DEFAULT_SQUARE_SIZE_UPPER_BOUND = 128   # v2/app_consts.go:5 (SquareSizeUpperBound)
TESTGROUND_SQUARE_SIZE_UPPER_BOUND = 512  # testground/app_consts.go:8
DEFAULT_GOV_MAX_SQUARE_SIZE = 64          # initial_consts.go:10
PARITY_SHARES_NAMESPACE = b"\xff" * 29                    # specs namespace.md:84
TAIL_PADDING_NAMESPACE = b"\xff" * 28 + b"\xfe"           # specs namespace.md:83
HASH_LENGTH = 32
SUBTREE_ROOT_THRESHOLD = 64             # v1/app_consts.go:6 (SubtreeRootThreshold, versioned_consts.go:21-23)
SHARE_VERSION_ZERO = 0
SUPPORTED_SHARE_VERSIONS = (SHARE_VERSION_ZERO,)  # global_consts.go:94-95
