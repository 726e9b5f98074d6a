"""Public constants of dplasma_amd.

Numeric values are identical to the reference's LAPACK-compatible enums
(``src/include/dplasma/constants.h:31-210``) so code written against the
reference's C API (or ScaLAPACK character arguments) maps 1:1.
"""
import torch

# --- error codes (constants.h:31-42)
DPLASMA_SUCCESS = 0
DPLASMA_ERR_NOT_INITIALIZED = -101
DPLASMA_ERR_REINITIALIZED = -102
DPLASMA_ERR_NOT_SUPPORTED = -103
DPLASMA_ERR_ILLEGAL_VALUE = -104
DPLASMA_ERR_NOT_FOUND = -105
DPLASMA_ERR_OUT_OF_RESOURCES = -106
DPLASMA_ERR_INTERNAL_LIMIT = -107
DPLASMA_ERR_UNALLOCATED = -108
DPLASMA_ERR_FILESYSTEM = -109
DPLASMA_ERR_UNEXPECTED = -110
DPLASMA_ERR_SEQUENCE_FLUSHED = -111

# --- precisions (constants.h:56-61)
dplasmaByte = 0
dplasmaInteger = 1
dplasmaRealFloat = 2
dplasmaRealDouble = 3
dplasmaComplexFloat = 4
dplasmaComplexDouble = 5

# --- layouts / BLAS enums (constants.h:73-100)
dplasmaRM = 101
dplasmaCM = 102
dplasmaNoTrans = 111
dplasmaTrans = 112
dplasmaConjTrans = 113
dplasmaUpper = 121
dplasmaLower = 122
dplasmaUpperLower = 123
dplasmaNonUnit = 131
dplasmaUnit = 132
dplasmaLeft = 141
dplasmaRight = 142
dplasmaOneNorm = 171
dplasmaRealOneNorm = 172
dplasmaTwoNorm = 173
dplasmaFrobeniusNorm = 174
dplasmaInfNorm = 175
dplasmaRealInfNorm = 176
dplasmaMaxNorm = 177
dplasmaRealMaxNorm = 178
dplasmaIncreasingOrder = 181
dplasmaDecreasingOrder = 182
dplasmaDistUniform = 201
dplasmaDistSymmetric = 202
dplasmaDistNormal = 203
dplasmaGeneral = 231
dplasmaSymmetric = 232
dplasmaHermitian = 233
dplasmaTriangular = 234
dplasmaLowerTriangular = 235
dplasmaUpperTriangular = 236
dplasmaNoVec = 301
dplasmaVec = 302
dplasmaIvec = 303
dplasmaAllVec = 304
dplasmaForward = 391
dplasmaBackward = 392
dplasmaColumnwise = 401
dplasmaRowwise = 402
dplasmaW = 501
dplasmaA2 = 502

# --- LAWN-263 test matrix generators (constants.h:163-207)
dplasmaMatrixRandom = 0
dplasmaMatrixHadamard = 1
dplasmaMatrixHouse = 2
dplasmaMatrixParter = 3
dplasmaMatrixRis = 4
dplasmaMatrixKms = 5
dplasmaMatrixToeppen = 6
dplasmaMatrixCondex = 7
dplasmaMatrixMoler = 8
dplasmaMatrixCircul = 9
dplasmaMatrixRandcorr = 10
dplasmaMatrixPoisson = 11
dplasmaMatrixHankel = 12
dplasmaMatrixJordbloc = 13
dplasmaMatrixCompan = 14
dplasmaMatrixPei = 15
dplasmaMatrixRandcolu = 16
dplasmaMatrixSprandn = 17
dplasmaMatrixRiemann = 18
dplasmaMatrixCompar = 19
dplasmaMatrixTridiag = 20
dplasmaMatrixChebspec = 21
dplasmaMatrixLehmer = 22
dplasmaMatrixToeppd = 23
dplasmaMatrixMinij = 24
dplasmaMatrixRandsvd = 25
dplasmaMatrixForsythe = 26
dplasmaMatrixFiedler = 27
dplasmaMatrixDorr = 28
dplasmaMatrixDemmel = 29
dplasmaMatrixChebvand = 30
dplasmaMatrixInvhess = 31
dplasmaMatrixProlate = 32
dplasmaMatrixFrank = 33
dplasmaMatrixCauchy = 34
dplasmaMatrixHilb = 35
dplasmaMatrixLotkin = 36
dplasmaMatrixKahan = 37
dplasmaMatrixOrthog = 38
dplasmaMatrixWilkinson = 39
dplasmaMatrixFoster = 40
dplasmaMatrixWright = 41
dplasmaMatrixLangou = 42

# --- storage of a tiled descriptor (tests/common.h:182-190)
STORAGE_TILE = "tile"
STORAGE_LAPACK = "lapack"

# --- precision letter <-> torch dtype <-> kernel code
PREC_DTYPE = {
    "s": torch.float32,
    "d": torch.float64,
    "c": torch.complex64,
    "z": torch.complex128,
}
DTYPE_PREC = {v: k for k, v in PREC_DTYPE.items()}
DTYPE_CODE = {
    torch.float32: dplasmaRealFloat,
    torch.float64: dplasmaRealDouble,
    torch.complex64: dplasmaComplexFloat,
    torch.complex128: dplasmaComplexDouble,
}
REAL_DTYPE = {
    torch.float32: torch.float32,
    torch.float64: torch.float64,
    torch.complex64: torch.float32,
    torch.complex128: torch.float64,
}

_LAPACK_CHAR = {
    dplasmaNoTrans: "N", dplasmaTrans: "T", dplasmaConjTrans: "C",
    dplasmaUpper: "U", dplasmaLower: "L", dplasmaUpperLower: "A",
    dplasmaNonUnit: "N", dplasmaUnit: "U", dplasmaLeft: "L", dplasmaRight: "R",
    dplasmaOneNorm: "O", dplasmaInfNorm: "I", dplasmaMaxNorm: "M", dplasmaFrobeniusNorm: "F",
}


def lapack_const(v: int) -> str:
    """Single LAPACK character for an enum (``dplasma_lapack_const``)."""
    return _LAPACK_CHAR[v]


_FROM_CHAR = {
    "trans": {"N": dplasmaNoTrans, "T": dplasmaTrans, "C": dplasmaConjTrans},
    "uplo": {"U": dplasmaUpper, "L": dplasmaLower, "A": dplasmaUpperLower, "G": dplasmaUpperLower},
    "diag": {"N": dplasmaNonUnit, "U": dplasmaUnit},
    "side": {"L": dplasmaLeft, "R": dplasmaRight},
    "norm": {"O": dplasmaOneNorm, "1": dplasmaOneNorm, "I": dplasmaInfNorm, "M": dplasmaMaxNorm,
             "F": dplasmaFrobeniusNorm, "E": dplasmaFrobeniusNorm},
}


def from_lapack_char(kind: str, c) -> int:
    """Map a ScaLAPACK character argument ('N', 'L', ...) to the enum; ints pass through."""
    if isinstance(c, int):
        return c
    return _FROM_CHAR[kind][str(c).upper()[0]]
