// Voronoi dust grid: the tessellation of a set of sites restricted to the domain box, and the queries
// the photon path needs. Reference: SKIRTcore/VoronoiDustGrid.cpp:28-138 (site generation),
// SKIRTcore/VoronoiMesh.cpp:250-306 (mesh and block lists), :512-541 (cellIndex), :591-618
// (randomPosition, isPointClosestTo), :749-844 (path). The reference computes the cells with the
// vendored Voro++ library; this is an independent implementation: every cell is the domain box clipped
// by the bisector planes of the sites near it, nearest first, until no farther site can cut it.
#pragma once

#include <functional>
#include <vector>

namespace skirt {

class UniformSource;

struct VoronoiGrid {
    double xmin = 0, xmax = 0, ymin = 0, ymax = 0, zmin = 0, zmax = 0;
    double eps = 0;                // 1e-12 * |extent widths| (VoronoiMesh constructor)
    std::vector<double> site;      // 3 per cell
    std::vector<int> nbrOffset;    // Ncells + 1
    std::vector<int> nbrList;      // neighbour cell indices; walls -1 xmin, -2 xmax, -3 ymin, -4 ymax, -5 zmin, -6 zmax
    std::vector<double> bbox;      // 6 per cell: xmin ymin zmin xmax ymax zmax of the cell's vertices
    std::vector<double> volume;    // per cell
    std::vector<double> centroid;  // 3 per cell
    // block lists accelerating cellIndex: nb^3 blocks over the domain, each listing the cells whose
    // (eps-widened) bounding box overlaps it
    int nb = 0;
    std::vector<int> blockOffset, blockList;

    int ncells() const { return (int)(site.size() / 3); }
    // the cell whose site is nearest to (x,y,z), or -1 outside the domain (VoronoiMesh::cellIndex)
    int cellIndex(double x, double y, double z) const;
    // VoronoiMesh::isPointClosestTo
    bool isPointClosestTo(double x, double y, double z, int m) const;
    // Box::cellindices for the block grid
    void blockIndices(double x, double y, double z, int& i, int& j, int& k) const;
};

// A node of the k-d tree over the sites that the cells' nearest-site queries use (leaves of at most 8
// sites perm[lo .. hi), split at the median of the widest axis; children after their parent)
struct KdNode {
    int lo, hi, left, right, dim;
    double split, bmin[3], bmax[3];
};

// The cells on another processor (skirt_mcrt_voronoi_cells on a HIP device): from the sites, the box
// {xmin, ymin, zmin, xmax, ymax, zmax} and the host's k-d tree, per cell its sorted neighbour ids (at most
// maxIds, at ids[i * maxIds]; nids[i] < 0: not computed, the host builds that cell), bounding box (6),
// volume and centroid (3), bit for bit as the host computes them. Throws on failure.
using VoronoiCellsFn = std::function<void(const std::vector<double>& sites, const double box[6],
                                          const std::vector<KdNode>& nodes, const std::vector<int>& perm, int maxIds,
                                          int* ids, int* nids, double* bbox, double* volume, double* centroid)>;

// builds the tessellation of `sites` (3 per site, all inside the box) in the box; with `cells`, the cells
// are computed there (the ones it leaves undone on the host), and *hostCells counts those the host built
void buildVoronoi(VoronoiGrid& g, const std::vector<double>& sites, double xmin, double xmax, double ymin,
                  double ymax, double zmin, double zmax, const VoronoiCellsFn* cells = nullptr,
                  int* hostCells = nullptr);

// VoronoiMesh::randomPosition: uniform points in the cell's bounding box until one lies in the cell
void voronoiRandomPosition(const VoronoiGrid& g, UniformSource& rng, int m, double& x, double& y, double& z);

}  // namespace skirt
