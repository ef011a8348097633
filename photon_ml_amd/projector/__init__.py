from .projectors import (IDENTITY, INDEX_MAP, IndexMapProjection, ProjectorKind, ProjectorType, RandomProjection,
                         gaussian_projection_matrix)

__all__ = ["IDENTITY", "INDEX_MAP", "IndexMapProjection", "ProjectorKind", "ProjectorType", "RandomProjection",
           "gaussian_projection_matrix"]
