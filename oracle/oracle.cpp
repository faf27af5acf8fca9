// CPU ORACLE -- test infrastructure only (see oracle.h). Restates the reference's photon life cycle.
#include "oracle.h"

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../skirt_amd/csrc/host/dustemission.hpp"
#include "../skirt_amd/csrc/host/model.hpp"
#include "../skirt_amd/csrc/host/outputs.hpp"

using namespace skirt;

namespace {

thread_local std::string g_error;

// ============================================================ random numbers

// Philox4x32-10 (Salmon et al. 2011, "Parallel random numbers: as easy as 1, 2, 3"), written out
// independently of the device engine's implementation so each can check the other.
void philox(const uint32_t in[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = in[0], c1 = in[1], c2 = in[2], c3 = in[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int round = 0; round < 10; round++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

class Rng {
public:
    virtual ~Rng() = default;
    virtual double uniform() = 0;
};

class MTRng final : public Rng {
public:
    explicit MTRng(MTRandom* mt) : mt_(mt) {}
    double uniform() override { return mt_->uniform(); }
private:
    MTRandom* mt_;
};

// one stream per packet: key = seed, counter = (block, tag, packet_lo, packet_hi); two 32-bit words
// make one 53-bit uniform in the open interval (0,1)
class PhiloxRng final : public Rng {
public:
    PhiloxRng(uint64_t seed, uint32_t tag) : tag_(tag) { key_[0] = (uint32_t)seed; key_[1] = (uint32_t)(seed >> 32); }
    void start(uint64_t packet) { packet_ = packet; block_ = 0; have_ = 0; }
    double uniform() override {
        if (have_ == 0) {
            uint32_t ctr[4] = {block_++, tag_, (uint32_t)packet_, (uint32_t)(packet_ >> 32)};
            philox(ctr, key_, w_);
            have_ = 4;
        }
        uint32_t a = w_[4 - have_], b = w_[5 - have_];
        have_ -= 2;
        uint64_t x = ((uint64_t)(a >> 5) << 26) | (uint64_t)(b >> 6);
        return ((double)x + 0.5) * (1.0 / 9007199254740992.0);
    }
private:
    uint32_t key_[2];
    uint32_t tag_;
    uint64_t packet_ = 0;
    uint32_t block_ = 0;
    uint32_t w_[4];
    int have_ = 0;
};

// Random::exponcutoff (Random.cpp:162-175)
double exponcutoff(Rng& r, double xmax) {
    if (xmax == 0.0) return 0.0;
    else if (xmax < 1e-10) return r.uniform() * xmax;
    double x = -log(1.0 - r.uniform() * (1.0 - exp(-xmax)));
    while (x > xmax) x = -log(1.0 - r.uniform() * (1.0 - exp(-xmax)));
    return x;
}

struct Vec3 { double x, y, z; };

// Direction(theta, phi) (Direction.cpp)
Vec3 directionThetaPhi(double theta, double phi) {
    const double eps = 1e-8;
    if (theta <= eps) return {0, 0, 1};
    if (theta >= M_PI - eps) return {0, 0, -1};
    double st = sin(theta);
    return {st * cos(phi), st * sin(phi), cos(theta)};
}

// Random::direction() (Random.cpp:179-184)
Vec3 isotropic(Rng& r) {
    double theta = acos(2.0 * r.uniform() - 1.0);
    double phi = 2.0 * M_PI * r.uniform();
    return directionThetaPhi(theta, phi);
}

// Random::direction(bfk, costheta) (Random.cpp:188-222)
Vec3 rotated(Rng& r, Vec3 k, double costheta) {
    double phi = 2.0 * M_PI * r.uniform();
    double cosphi = cos(phi), sinphi = sin(phi);
    double sintheta = sqrt(fabs((1.0 - costheta) * (1.0 + costheta)));
    double kx = k.x, ky = k.y, kz = k.z;
    if (kz > 0.99999) return {cosphi * sintheta, sinphi * sintheta, costheta};
    if (kz < -0.99999) return {cosphi * sintheta, sinphi * sintheta, -costheta};
    double root = sqrt((1.0 - kz) * (1.0 + kz));
    return {sintheta / root * (-kx * kz * cosphi + ky * sinphi) + kx * costheta,
            -sintheta / root * (ky * kz * cosphi + kx * sinphi) + ky * costheta,
            root * sintheta * cosphi + kz * costheta};
}

// ============================================================ paths

struct Segment { int m; double ds, s, dtau, tau; };

struct Path {
    std::vector<Segment> v;
    double s = 0;
    void clear() { v.clear(); s = 0; }
    void add(int m, double ds) {  // DustGridPath::addSegment
        if (ds > 0) { s += ds; v.push_back({m, ds, s, 0, 0}); }
    }
};

// CartesianDustGrid::path (CartesianDustGrid.cpp:136-283)
void cartesianPath(const CartesianGrid& g, Vec3 r, Vec3 k, Path& p) {
    p.clear();
    double kx = k.x, ky = k.y, kz = k.z, x = r.x, y = r.y, z = r.z, ds, dsx, dsy, dsz;
    const std::vector<double>&xv = g.xv, &yv = g.yv, &zv = g.zv;
    if (x < g.xmin) {
        if (kx <= 0.0) return p.clear();
        ds = (g.xmin - x) / kx; p.add(-1, ds);
        x = g.xmin + 1e-8 * (xv[1] - xv[0]); y += ky * ds; z += kz * ds;
    } else if (x > g.xmax) {
        if (kx >= 0.0) return p.clear();
        ds = (g.xmax - x) / kx; p.add(-1, ds);
        x = g.xmax - 1e-8 * (xv[g.Nx] - xv[g.Nx - 1]); y += ky * ds; z += kz * ds;
    }
    if (y < g.ymin) {
        if (ky <= 0.0) return p.clear();
        ds = (g.ymin - y) / ky; p.add(-1, ds);
        x += kx * ds; y = g.ymin + 1e-8 * (yv[1] - yv[0]); z += kz * ds;
    } else if (y > g.ymax) {
        if (ky >= 0.0) return p.clear();
        ds = (g.ymax - y) / ky; p.add(-1, ds);
        x += kx * ds; y = g.ymax - 1e-8 * (yv[g.Ny] - yv[g.Ny - 1]); z += kz * ds;
    }
    if (z < g.zmin) {
        if (kz <= 0.0) return p.clear();
        ds = (g.zmin - z) / kz; p.add(-1, ds);
        x += kx * ds; y += ky * ds; z = g.zmin + 1e-8 * (zv[1] - zv[0]);
    } else if (z > g.zmax) {
        if (kz >= 0.0) return p.clear();
        ds = (g.zmax - z) / kz; p.add(-1, ds);
        x += kx * ds; y += ky * ds; z = g.zmax - 1e-8 * (zv[g.Nz] - zv[g.Nz - 1]);
    }
    if (x < g.xmin || x > g.xmax || y < g.ymin || y > g.ymax || z < g.zmin || z > g.zmax) return p.clear();
    auto clip = [](const std::vector<double>& v, double q) {  // NR::locate_clip
        int n = (int)v.size();
        if (q < v[0]) return 0;
        int jl = -1, ju = n - 1;
        while (ju - jl > 1) { int jm = (ju + jl) >> 1; if (q < v[jm]) ju = jm; else jl = jm; }
        return jl;
    };
    int i = clip(xv, x), j = clip(yv, y), kk = clip(zv, z);
    while (true) {
        int m = kk + g.Nz * j + g.Nz * g.Ny * i;
        double xE = (kx < 0.0) ? xv[i] : xv[i + 1];
        double yE = (ky < 0.0) ? yv[j] : yv[j + 1];
        double zE = (kz < 0.0) ? zv[kk] : zv[kk + 1];
        dsx = (fabs(kx) > 1e-15) ? (xE - x) / kx : DBL_MAX;
        dsy = (fabs(ky) > 1e-15) ? (yE - y) / ky : DBL_MAX;
        dsz = (fabs(kz) > 1e-15) ? (zE - z) / kz : DBL_MAX;
        if (dsx <= dsy && dsx <= dsz) {
            ds = dsx; p.add(m, ds);
            i += (kx < 0.0) ? -1 : 1;
            if (i >= g.Nx || i < 0) return;
            x = xE; y += ky * ds; z += kz * ds;
        } else if (dsy < dsx && dsy <= dsz) {
            ds = dsy; p.add(m, ds);
            j += (ky < 0.0) ? -1 : 1;
            if (j >= g.Ny || j < 0) return;
            x += kx * ds; y = yE; z += kz * ds;
        } else if (dsz < dsx && dsz < dsy) {
            ds = dsz; p.add(m, ds);
            kk += (kz < 0.0) ? -1 : 1;
            if (kk >= g.Nz || kk < 0) return;
            x += kx * ds; y += ky * ds; z = zE;
        } else {
            return;  // NaN guard: the reference would loop forever here
        }
    }
}


// DustGridPath::moveInside (DustGridPath.cpp:57-150) for a box {xmin ymin zmin xmax ymax zmax}: the
// segments outside the box (m = -1) and the entry point, or infinity when the path misses the box
void moveInsideBox(const double* b, double eps, Vec3 k, Path& p, double& rx, double& ry, double& rz) {
    double kx = k.x, ky = k.y, kz = k.z;
    bool outside = false;
    if (rx <= b[0]) {
        if (kx <= 0.0) outside = true;
        else { double ds = (b[0] - rx) / kx; p.add(-1, ds); rx = b[0] + eps; ry += ky * ds; rz += kz * ds; }
    } else if (rx >= b[3]) {
        if (kx >= 0.0) outside = true;
        else { double ds = (b[3] - rx) / kx; p.add(-1, ds); rx = b[3] - eps; ry += ky * ds; rz += kz * ds; }
    }
    if (!outside) {
        if (ry <= b[1]) {
            if (ky <= 0.0) outside = true;
            else { double ds = (b[1] - ry) / ky; p.add(-1, ds); rx += kx * ds; ry = b[1] + eps; rz += kz * ds; }
        } else if (ry >= b[4]) {
            if (ky >= 0.0) outside = true;
            else { double ds = (b[4] - ry) / ky; p.add(-1, ds); rx += kx * ds; ry = b[4] - eps; rz += kz * ds; }
        }
    }
    if (!outside) {
        if (rz <= b[2]) {
            if (kz <= 0.0) outside = true;
            else { double ds = (b[2] - rz) / kz; p.add(-1, ds); rx += kx * ds; ry += ky * ds; rz = b[2] + eps; }
        } else if (rz >= b[5]) {
            if (kz >= 0.0) outside = true;
            else { double ds = (b[5] - rz) / kz; p.add(-1, ds); rx += kx * ds; ry += ky * ds; rz = b[5] - eps; }
        }
    }
    if (outside) { rx = ry = rz = INFINITY; }
}

// VoronoiMesh::path (VoronoiMesh.cpp:749-844): from the current cell, the nearest positive crossing of
// the bisector planes with its neighbours (or of the domain walls)
void voronoiPath(const VoronoiGrid& g, Vec3 r0, Vec3 k, Path& p) {
    p.clear();
    const double box[6] = {g.xmin, g.ymin, g.zmin, g.xmax, g.ymax, g.zmax};
    double rx = r0.x, ry = r0.y, rz = r0.z;
    moveInsideBox(box, g.eps, k, p, rx, ry, rz);
    int mr = g.cellIndex(rx, ry, rz);
    if (mr < 0) return p.clear();
    const double* S = g.site.data();
    long guard = 0;
    while (mr >= 0) {
        if (++guard > 10000000)
            throw std::runtime_error("Voronoi path does not advance: cell " + std::to_string(mr) + " at (" +
                                     std::to_string(rx) + "," + std::to_string(ry) + "," + std::to_string(rz) + ") k (" +
                                     std::to_string(k.x) + "," + std::to_string(k.y) + "," + std::to_string(k.z) + ")");
        const double prx = S[3 * mr], pry = S[3 * mr + 1], prz = S[3 * mr + 2];
        double sq = DBL_MAX;
        const int NO_INDEX = -99;
        int mq = NO_INDEX;
        for (int q = g.nbrOffset[mr]; q < g.nbrOffset[mr + 1]; q++) {
            const int mi = g.nbrList[q];
            double si = 0;
            if (mi >= 0) {
                const double pix = S[3 * mi], piy = S[3 * mi + 1], piz = S[3 * mi + 2];
                const double nx = pix - prx, ny = piy - pry, nz = piz - prz;
                const double ndotk = nx * k.x + ny * k.y + nz * k.z;
                if (ndotk > 0) {
                    const double px = 0.5 * (pix + prx), py = 0.5 * (piy + pry), pz = 0.5 * (piz + prz);
                    si = (nx * (px - rx) + ny * (py - ry) + nz * (pz - rz)) / ndotk;
                }
            } else {
                switch (mi) {
                case -1: si = (g.xmin - rx) / k.x; break;
                case -2: si = (g.xmax - rx) / k.x; break;
                case -3: si = (g.ymin - ry) / k.y; break;
                case -4: si = (g.ymax - ry) / k.y; break;
                case -5: si = (g.zmin - rz) / k.z; break;
                case -6: si = (g.zmax - rz) / k.z; break;
                default: throw std::runtime_error("Invalid neighbor ID");
                }
            }
            if (si > 0 && si < sq) { sq = si; mq = mi; }
        }
        if (mq == NO_INDEX) {
            rx += k.x * g.eps; ry += k.y * g.eps; rz += k.z * g.eps;
            mr = g.cellIndex(rx, ry, rz);
        } else {
            p.add(mr, sq);
            rx += (sq + g.eps) * k.x; ry += (sq + g.eps) * k.y; rz += (sq + g.eps) * k.z;
            mr = mq;
        }
    }
}

// TreeNode::whichnode(r) from the root (TreeNode.cpp:70-80), OctTreeNode::child(r) / BinTreeNode::child(r)
int rootWhichnode(const OctreeGrid& t, double x, double y, double z) {
    const double* b = &t.box[0];
    if (!(x >= b[0] && x <= b[3] && y >= b[1] && y <= b[4] && z >= b[2] && z <= b[5])) return -1;
    int l = 0;
    while (t.firstChild[l] >= 0) l = t.child(l, x, y, z);
    return l;
}

// TreeDustGrid::path, Bookkeeping search (TreeDustGrid.cpp:523-659): octrees only; the next node comes
// from the breadth-first numbering (children of a node are 8 consecutive ids in octant order, so
// (l-1) % 8 is a node's octant): climb while the node lies on the far side of its father, step to the
// sibling across the wall, descend with "<=" to the leaf holding the exit point. No eps nudge: the
// position is put on the crossed wall exactly.
void bookkeepingPath(const OctreeGrid& t, int l, double x, double y, double z, double kx, double ky, double kz,
                     Path& p) {
    auto B = [&](int n) { return &t.box[6 * (size_t)n]; };
    auto child = [&](int n, int k) { return t.firstChild[n] + k; };
    while (true) {
        const double* b = B(l);
        double xnext = (kx < 0.0) ? b[0] : b[3];
        double ynext = (ky < 0.0) ? b[1] : b[4];
        double znext = (kz < 0.0) ? b[2] : b[5];
        double dsx = (fabs(kx) > 1e-15) ? (xnext - x) / kx : DBL_MAX;
        double dsy = (fabs(ky) > 1e-15) ? (ynext - y) / ky : DBL_MAX;
        double dsz = (fabs(kz) > 1e-15) ? (znext - z) / kz : DBL_MAX;
        if (dsx <= dsy && dsx <= dsz) {
            p.add(t.cellnumber[l], dsx);
            x = xnext; y += ky * dsx; z += kz * dsx;
            while (true) {
                int oct = ((l - 1) % 8) + 1;
                bool place = (kx < 0.0) ? (oct % 2 == 1) : (oct % 2 == 0);
                if (!place) break;
                l = t.father[l];
                if (l == 0) return;
            }
            l += (kx < 0.0) ? -1 : 1;
            while (t.cellnumber[l] == -1) {
                double yM = B(child(l, 0))[4], zM = B(child(l, 0))[5];
                if (kx < 0.0) l = (y <= yM) ? ((z <= zM) ? child(l, 1) : child(l, 5)) : ((z <= zM) ? child(l, 3) : child(l, 7));
                else l = (y <= yM) ? ((z <= zM) ? child(l, 0) : child(l, 4)) : ((z <= zM) ? child(l, 2) : child(l, 6));
            }
        } else if (dsy < dsx && dsy <= dsz) {
            p.add(t.cellnumber[l], dsy);
            x += kx * dsy; y = ynext; z += kz * dsy;
            while (true) {
                bool place = (ky < 0.0) ? ((l - 1) % 4 < 2) : ((l - 1) % 4 > 1);
                if (!place) break;
                l = t.father[l];
                if (l == 0) return;
            }
            l += (ky < 0.0) ? -2 : 2;
            while (t.cellnumber[l] == -1) {
                double xM = B(child(l, 0))[3], zM = B(child(l, 0))[5];
                if (ky < 0.0) l = (x <= xM) ? ((z <= zM) ? child(l, 2) : child(l, 6)) : ((z <= zM) ? child(l, 3) : child(l, 7));
                else l = (x <= xM) ? ((z <= zM) ? child(l, 0) : child(l, 4)) : ((z <= zM) ? child(l, 1) : child(l, 5));
            }
        } else if (dsz < dsx && dsz < dsy) {
            p.add(t.cellnumber[l], dsz);
            x += kx * dsz; y += ky * dsz; z = znext;
            while (true) {
                int oct = ((l - 1) % 8) + 1;
                bool place = (kz < 0.0) ? (oct < 5) : (oct > 4);
                if (!place) break;
                l = t.father[l];
                if (l == 0) return;
            }
            l += (kz < 0.0) ? -4 : 4;
            while (t.cellnumber[l] == -1) {
                double xM = B(child(l, 0))[3], yM = B(child(l, 0))[4];
                if (kz < 0.0) l = (x <= xM) ? ((y <= yM) ? child(l, 4) : child(l, 6)) : ((y <= yM) ? child(l, 5) : child(l, 7));
                else l = (x <= xM) ? ((y <= yM) ? child(l, 0) : child(l, 2)) : ((y <= yM) ? child(l, 1) : child(l, 3));
            }
        } else {
            return;  // NaN distances: the reference would loop forever; end the path
        }
    }
}

// TreeDustGrid::path, TopDown and Neighbor search (TreeDustGrid.cpp:390-521); moveInside
// (DustGridPath.cpp:57-150)
void octreePath(const OctreeGrid& t, Vec3 r, Vec3 k, Path& p) {
    p.clear();
    double kx = k.x, ky = k.y, kz = k.z, rx = r.x, ry = r.y, rz = r.z;
    const double eps = t.eps;
    const double bx0 = t.box[0], by0 = t.box[1], bz0 = t.box[2], bx1 = t.box[3], by1 = t.box[4], bz1 = t.box[5];
    // moveInside
    {
        bool outside = false;
        if (rx <= bx0) {
            if (kx <= 0.0) outside = true;
            else { double ds = (bx0 - rx) / kx; p.add(-1, ds); rx = bx0 + eps; ry += ky * ds; rz += kz * ds; }
        } else if (rx >= bx1) {
            if (kx >= 0.0) outside = true;
            else { double ds = (bx1 - rx) / kx; p.add(-1, ds); rx = bx1 - eps; ry += ky * ds; rz += kz * ds; }
        }
        if (!outside) {
            if (ry <= by0) {
                if (ky <= 0.0) outside = true;
                else { double ds = (by0 - ry) / ky; p.add(-1, ds); rx += kx * ds; ry = by0 + eps; rz += kz * ds; }
            } else if (ry >= by1) {
                if (ky >= 0.0) outside = true;
                else { double ds = (by1 - ry) / ky; p.add(-1, ds); rx += kx * ds; ry = by1 - eps; rz += kz * ds; }
            }
        }
        if (!outside) {
            if (rz <= bz0) {
                if (kz <= 0.0) outside = true;
                else { double ds = (bz0 - rz) / kz; p.add(-1, ds); rx += kx * ds; ry += ky * ds; rz = bz0 + eps; }
            } else if (rz >= bz1) {
                if (kz >= 0.0) outside = true;
                else { double ds = (bz1 - rz) / kz; p.add(-1, ds); rx += kx * ds; ry += ky * ds; rz = bz1 - eps; }
            }
        }
        if (outside) { rx = ry = rz = INFINITY; }
    }
    int node = rootWhichnode(t, rx, ry, rz);
    if (node < 0) return p.clear();
    double x = rx, y = ry, z = rz;
    if (t.search == 2) return bookkeepingPath(t, node, x, y, z, kx, ky, kz, p);
    while (node >= 0) {
        const double* b = &t.box[6 * (size_t)node];
        double xnext = (kx < 0.0) ? b[0] : b[3];
        double ynext = (ky < 0.0) ? b[1] : b[4];
        double znext = (kz < 0.0) ? b[2] : b[5];
        double dsx = (fabs(kx) > 1e-15) ? (xnext - x) / kx : DBL_MAX;
        double dsy = (fabs(ky) > 1e-15) ? (ynext - y) / ky : DBL_MAX;
        double dsz = (fabs(kz) > 1e-15) ? (znext - z) / kz : DBL_MAX;
        double ds;
        int wall;
        if (dsx <= dsy && dsx <= dsz) { ds = dsx; wall = (kx < 0.0) ? 0 : 1; }
        else if (dsy <= dsx && dsy <= dsz) { ds = dsy; wall = (ky < 0.0) ? 2 : 3; }
        else { ds = dsz; wall = (kz < 0.0) ? 4 : 5; }
        p.add(t.cellnumber[node], ds);
        x += (ds + eps) * kx;
        y += (ds + eps) * ky;
        z += (ds + eps) * kz;
        int oldnode = node;
        if (t.search == 0) {
            node = rootWhichnode(t, x, y, z);
        } else {
            node = -1;
            size_t q = 6 * (size_t)oldnode + wall;
            for (int n = t.nbrOffset[q]; n < t.nbrOffset[q + 1]; n++) {
                int c = t.nbrList[n];
                const double* cb = &t.box[6 * (size_t)c];
                if (x >= cb[0] && x <= cb[3] && y >= cb[1] && y <= cb[4] && z >= cb[2] && z <= cb[5]) { node = c; break; }
            }
            if (node < 0) node = rootWhichnode(t, x, y, z);
        }
        if (node == oldnode) {
            x = nextafter(x, (kx < 0.0) ? -DBL_MAX : DBL_MAX);
            y = nextafter(y, (ky < 0.0) ? -DBL_MAX : DBL_MAX);
            z = nextafter(z, (kz < 0.0) ? -DBL_MAX : DBL_MAX);
            node = rootWhichnode(t, x, y, z);
            if (node == oldnode) break;
        }
    }
}

// ============================================================ simulation

// LockFree::add (Fundamentals/LockFree.hpp:25-37): compare-and-swap loop on a double
inline void lockFreeAdd(double* p, double v) {
    uint64_t* q = reinterpret_cast<uint64_t*>(p);
    uint64_t cur = __atomic_load_n(q, __ATOMIC_RELAXED);
    while (true) {
        double d;
        std::memcpy(&d, &cur, 8);
        d += v;
        uint64_t nw;
        std::memcpy(&nw, &d, 8);
        if (__atomic_compare_exchange_n(q, &cur, nw, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) return;
    }
}

constexpr size_t kCrossedBins = 1 << 16;

// Test switch (oracle_set_engine_attenuation): how exp(-tau_{n-1}) of the absorption sum is evaluated.
//   0 the reference's exp(-taustart) per segment (MonteCarloSimulation.cpp:458-462), the default;
//   1 the running product of 1 - (-expm1(-dtau)) over the path's dust segments, as the GPU engine carried it
//     until round 3. It parts from 0 in the last digits only behind optically thick segments, where
//     1 - (1 - exp(-dtau)) cancels: tests/test_attenuation.py shows that this was the whole of the engine's
//     deep-cell differences on thick models then;
//   2 the engine's carry since round 5 (Tracer::segment, engine.hip): f <- f - f * (-expm1(-dtau)) while
//     dtau < 0.5 (kCarryTau), exp(-tau_n) evaluated anew after a thicker segment.
static std::atomic<int> g_engineAttenuation{0};
static int engineAttenuation() { return g_engineAttenuation.load(std::memory_order_relaxed); }
constexpr double kEngineCarryTau = 0.5;  // engine.hip kCarryTau
// the next segment's exp(-tau_{n-1}) factor after segment n (dtau, cumulative tau), in mode `mode`
static inline double nextAttenuation(int mode, double att, double expfactorm, double dtau, double tau) {
    if (mode == 2) return dtau < kEngineCarryTau ? att - att * expfactorm : exp(-tau);
    return att * (1.0 - expfactorm);
}

// diagnostic (tools/parity_trace.py): ORACLE_DEBUG_FILL=1 prints every storing one-component FILL path (start,
// direction, luminosity) and its dust segments (cell, ds, dtau, Labs add) to stdout; run single-threaded
static bool debugFill() {
    static const bool on = getenv("ORACLE_DEBUG_FILL") && atoi(getenv("ORACLE_DEBUG_FILL")) != 0;
    return on;
}

// study hook (oracle_set_fill_hook): the cells of every storing FILL path
static OracleFillHook g_fillHook = nullptr;
static void* g_fillUser = nullptr;

struct Tallies {
    bool shared = false;       // threaded mode: one set of arrays updated with lock-free adds
    void add(std::vector<double>& v, size_t i, double x) {
        if (shared) lockFreeAdd(&v[i], x);
        else v[i] += x;
    }
    std::vector<double> labs;  // Ncells x Nlambda row-major (stellar)
    std::vector<double> labsDust;
    std::vector<std::vector<double>> frames, seds;  // per instrument
    std::atomic<uint64_t> segments{0};
    // the counts behind the engine's statistics: segments of the FILL paths (fillOpticalDepth) and of the
    // peel-off paths (opticaldepth), Labs adds; and DustSystem's _crossed histogram (DustSystem.cpp:959-1000):
    // paths per number of segments (cells crossed, including those outside the grid), last bin = overflow
    std::atomic<uint64_t> segFill{0}, segPeel{0}, absorbs{0};
    std::vector<uint64_t> crossed = std::vector<uint64_t>(kCrossedBins, 0);
};

// The counts above, kept per thread while a phase runs and added to the Tallies when the thread ends: a
// shared atomic per path or per absorbing segment would serialize the worker threads (the CPU baseline
// of bench.py runs on this code).
struct Counts {
    uint64_t segments = 0, segFill = 0, segPeel = 0, absorbs = 0;
    std::vector<uint64_t> crossed = std::vector<uint64_t>(kCrossedBins, 0);
    void cross(size_t n) { crossed[std::min(n, crossed.size() - 1)]++; }
    void mergeInto(Tallies& t) const {
        t.segments.fetch_add(segments);
        t.segFill.fetch_add(segFill);
        t.segPeel.fetch_add(segPeel);
        t.absorbs.fetch_add(absorbs);
        for (size_t i = 0; i < crossed.size(); i++)
            if (crossed[i]) __atomic_fetch_add(&t.crossed[i], crossed[i], __ATOMIC_RELAXED);
    }
};
thread_local Counts* tCounts = nullptr;
inline Counts& counts() {
    static thread_local Counts spare;  // calls outside a phase (none on the hot path)
    return tCounts ? *tCounts : spare;
}

class Sim {
public:
    Sim(const Model& m) : M(m) {}

    const Model& M;

    void path(Vec3 r, Vec3 k, Path& p) const {
        if (M.grid.kind == GridKind::Cartesian) cartesianPath(M.grid.cart, r, k, p);
        else if (M.grid.kind == GridKind::Voronoi) voronoiPath(M.grid.vor, r, k, p);
        else {
            octreePath(M.grid.tree, r, k, p);
        }
    }

    void initTallies(Tallies& t) const {
        if (M.hasDust && M.storeAbsorption) t.labs.assign((size_t)M.ncells() * M.wl.n(), 0.0);
        t.frames.resize(M.instruments.size());
        t.seds.resize(M.instruments.size());
        for (size_t i = 0; i < M.instruments.size(); i++) {
            const Instrument& ins = M.instruments[i];
            if (ins.hasFrames()) t.frames[i].assign((size_t)ins.nslots() * M.wl.n() * ins.nframe(), 0.0);
            if (ins.hasSeds()) t.seds[i].assign((size_t)ins.nslots() * M.wl.n(), 0.0);
        }
    }

    struct Packet {
        double L;
        int ell;
        Vec3 r, k;
        int nscatt;
        int stellar;  // component index, or -1 for dust emission
    };

    // Instrument::detect for the four distant-instrument kinds
    void detect(Tallies& t, int i, const Packet& pp, Path& tmp) const {
        const Instrument& ins = M.instruments[i];
        int nscatt = pp.nscatt, ell = pp.ell, Nl = M.wl.n();
        double L = pp.L;
        int l = ins.kind == InstrumentKind::SED ? -1 : ins.pixel(pp.r.x, pp.r.y, pp.r.z);
        if (ins.kind == InstrumentKind::Frame && l < 0) return;
        double taupath = 0;
        if (M.hasDust) {
            Vec3 ko{ins.kobs[0], ins.kobs[1], ins.kobs[2]};
            path(pp.r, ko, tmp);
            Counts& c = counts();
            c.segments += tmp.v.size();
            c.segPeel += tmp.v.size();
            c.cross(tmp.v.size());
            for (auto& s : tmp.v) taupath += M.kapparho(s.m, ell) * s.ds;
        }
        double extf = exp(-taupath);
        double Lextf = L * extf;
        auto sed = [&](int slot, double v) { t.add(t.seds[i], (size_t)slot * Nl + ell, v); };
        auto frm = [&](int slot, double v) {
            if (l >= 0) t.add(t.frames[i], ((size_t)slot * Nl + ell) * ins.nframe() + l, v);
        };
        if (ins.kind != InstrumentKind::Full) {
            if (ins.hasSeds()) sed(0, Lextf);
            if (ins.hasFrames()) frm(0, Lextf);
            return;
        }
        for (int pass = 0; pass < 2; pass++) {
            auto add = [&](int slot, double v) { if (pass == 0) sed(slot, v); else frm(slot, v); };
            if (pp.stellar >= 0) {
                if (nscatt == 0) {
                    add(SlotTrav, L);
                    if (M.hasDust) add(SlotStrDir, Lextf);
                } else {
                    add(SlotStrSca, Lextf);
                    if (nscatt <= ins.scatteringLevels) add(SlotLevel0 + nscatt - 1, Lextf);
                }
            } else {
                if (nscatt == 0) add(SlotDusDir, Lextf);
                else add(SlotDusSca, Lextf);
            }
        }
    }

    // MonteCarloSimulation::continuouspeeloffscattering (MonteCarloSimulation.cpp:367-434), unpolarized:
    // from a uniformly drawn point of every path segment with scattering dust, a peel-off toward every
    // instrument weighted by the luminosity scattered in the segment
    void continuousPeelOff(Tallies& t, Rng& rng, const Packet& pp, const Path& p, Path& tmp) const {
        const int Ncomp = M.ncomp();
        const int ell = pp.ell;
        double wv[16];
        const int N = (int)p.v.size();
        for (int n = 0; n < N; n++) {
            const int m = p.v[n].m;
            if (m == -1) continue;
            double ksca = 0.0, kext = 0.0;
            for (int h = 0; h < Ncomp; h++) {
                const double rho = M.rho[(size_t)m * Ncomp + h];
                wv[h] = rho * M.dust[h].mix.ksca[ell];
                ksca += rho * M.dust[h].mix.ksca[ell];
                kext += rho * M.dust[h].mix.kext[ell];
            }
            if (!(ksca > 0.0)) continue;
            for (int h = 0; h < Ncomp; h++) wv[h] /= ksca;
            const double albedo = ksca / kext;
            const double tau0 = (n == 0) ? 0.0 : p.v[n - 1].tau;
            const double dtau = p.v[n].dtau;
            const double s0 = (n == 0) ? 0.0 : p.v[n - 1].s;
            const double ds = p.v[n].ds;
            const double factorm = albedo * exp(-tau0) * (-expm1(-dtau));
            const double s = s0 + rng.uniform() * ds;
            const Vec3 rnew{pp.r.x + s * pp.k.x, pp.r.y + s * pp.k.y, pp.r.z + s * pp.k.z};
            for (size_t i = 0; i < M.instruments.size(); i++) {
                const Instrument& ins = M.instruments[i];
                double I = 0;
                for (int h = 0; h < Ncomp; h++) {
                    const double cosalpha = pp.k.x * ins.kobs[0] + pp.k.y * ins.kobs[1] + pp.k.z * ins.kobs[2];
                    const double g = M.dust[h].mix.g[ell];
                    const double tt = 1.0 + g * g - 2 * g * cosalpha;
                    const double w = wv[h] * ((1.0 - g) * (1.0 + g) / sqrt(tt * tt * tt));
                    I += w * 1.0;
                }
                Packet ppp = pp;  // PhotonPackage::launchScatteringPeelOff(pp, bfrnew, bfkobs, factorm*I)
                ppp.L = pp.L * (factorm * I);
                ppp.r = rnew;
                ppp.k = {ins.kobs[0], ins.kobs[1], ins.kobs[2]};
                ppp.nscatt = pp.nscatt + 1;
                detect(t, (int)i, ppp, tmp);
            }
        }
    }

    // the photon life cycle after launch: MonteCarloSimulation.cpp:283-293
    void lifeCycle(Tallies& t, Rng& rng, Packet& pp, double Lthreshold, bool peel, bool store,
                   std::vector<double>* labs, Path& p, Path& tmp) const {
        int Ncomp = M.ncomp();
        int Nl = M.wl.n();
        if (peel)
            for (size_t i = 0; i < M.instruments.size(); i++) detect(t, (int)i, pp, tmp);  // peeloffemission
        while (true) {
            // DustSystem::fillOpticalDepth
            path(pp.r, pp.k, p);
            Counts& c = counts();
            c.segments += p.v.size();
            c.segFill += p.v.size();
            c.cross(p.v.size());
            double tau = 0;
            for (auto& s : p.v) {
                double dtau = M.kapparho(s.m, pp.ell) * s.ds;
                tau += dtau;
                s.dtau = dtau;
                s.tau = tau;
            }
            double taupath = p.v.empty() ? 0 : p.v.back().tau;
            if (taupath < 0.0 || std::isnan(taupath) || std::isinf(taupath))
                throw std::runtime_error("the optical depth along the path is not a positive number");
            if (peel && M.continuousScattering) continuousPeelOff(t, rng, pp, p, tmp);
            if (g_fillHook && store) {
                std::vector<int> cells;
                for (auto& s : p.v)
                    if (s.m != -1) cells.push_back(s.m);
                const double r0[3] = {pp.r.x, pp.r.y, pp.r.z}, k0[3] = {pp.k.x, pp.k.y, pp.k.z};
                g_fillHook(g_fillUser, pp.ell, r0, k0, cells.data(), (int)cells.size());
            }
            // simulateescapeandabsorption
            double L = pp.L;
            if (Ncomp == 1) {
                double albedo = M.dust[0].mix.albedo[pp.ell];
                double expfactor = -expm1(-taupath);
                if (store) {
                    int N = (int)p.v.size();
                    const int mode = engineAttenuation();
                    double att = 1.0;  // (modes 1, 2) exp(-taustart) as the engine carries it
                    if (debugFill())
                        printf("O L %d %.17g %.17g %.17g %.17g %.17g %.17g %.17g\n", pp.ell, pp.r.x, pp.r.y, pp.r.z,
                               pp.k.x, pp.k.y, pp.k.z, L);
                    for (int n = 0; n < N; n++) {
                        int m = p.v[n].m;
                        if (m != -1) {
                            double taustart = (n == 0) ? 0.0 : p.v[n - 1].tau;
                            double expfactorm = -expm1(-p.v[n].dtau);
                            double Lintm = L * (mode ? att : exp(-taustart)) * expfactorm;
                            att = nextAttenuation(mode, att, expfactorm, p.v[n].dtau, p.v[n].tau);
                            double Labsm = (1.0 - albedo) * Lintm;
                            if (debugFill()) printf("O S %d %.17g %.17g %.17g\n", m, p.v[n].ds, p.v[n].dtau, Labsm);
                            t.add(*labs, (size_t)m * Nl + pp.ell, Labsm);
                            counts().absorbs++;
                        }
                    }
                }
                pp.L = L * albedo * expfactor;
            } else {
                double Lsca = 0.0;
                int N = (int)p.v.size();
                const int mode = engineAttenuation();
                double att = 1.0;
                for (int n = 0; n < N; n++) {
                    int m = p.v[n].m;
                    if (m != -1) {
                        double ksca = 0.0, kext = 0.0;
                        for (int h = 0; h < Ncomp; h++) {
                            double rho = M.rho[(size_t)m * Ncomp + h];
                            ksca += rho * M.dust[h].mix.ksca[pp.ell];
                            kext += rho * M.dust[h].mix.kext[pp.ell];
                        }
                        double albedo = (kext > 0.0) ? ksca / kext : 0.0;
                        double taustart = (n == 0) ? 0.0 : p.v[n - 1].tau;
                        double expfactorm = -expm1(-p.v[n].dtau);
                        double Lintm = L * (mode ? att : exp(-taustart)) * expfactorm;
                        att = nextAttenuation(mode, att, expfactorm, p.v[n].dtau, p.v[n].tau);
                        Lsca += albedo * Lintm;
                        if (store) {
                            t.add(*labs, (size_t)m * Nl + pp.ell, (1.0 - albedo) * Lintm);
                            counts().absorbs++;
                        }
                    }
                }
                pp.L = Lsca;
            }
            if (pp.L <= 0 || (pp.L <= Lthreshold && pp.nscatt >= M.minScattEvents)) break;
            // simulatepropagation
            if (taupath != 0.0) {
                double tauint;
                double xi = M.scattBias;
                if (xi == 0.0) tauint = exponcutoff(rng, taupath);
                else {
                    double X = rng.uniform();
                    tauint = (X < xi) ? rng.uniform() * taupath : exponcutoff(rng, taupath);
                    double pr = -exp(-tauint) / expm1(-taupath);
                    double q = (1.0 - xi) * pr + xi / taupath;
                    double weight = pr / q;
                    pp.L = pp.L * weight;
                }
                // DustGridPath::pathlength (DustGridPath.cpp:162-173) with NR::locate on the tau column
                double s = 0;
                int N = (int)p.v.size();
                if (N > 0 && tauint > 0) {
                    int i;
                    if (tauint < p.v[0].tau) i = -1;
                    else if (p.v[N - 1].tau < tauint) i = N - 1;
                    else {
                        int jl = -1, ju = N;
                        while (ju - jl > 1) { int jm = (ju + jl) >> 1; if (tauint < p.v[jm].tau) ju = jm; else jl = jm; }
                        i = (jl <= 0) ? 0 : (jl >= N - 2) ? N - 2 : jl;
                    }
                    auto lin = [](double x, double x1, double x2, double f1, double f2) { return f1 + ((x - x1) / (x2 - x1)) * (f2 - f1); };
                    if (i < 0) s = lin(tauint, 0, p.v[0].tau, 0, p.v[0].s);
                    else if (i < N - 1) s = lin(tauint, p.v[i].tau, p.v[i + 1].tau, p.v[i].s, p.v[i + 1].s);
                    else s = p.v[N - 1].s;
                }
                pp.r = {pp.r.x + s * pp.k.x, pp.r.y + s * pp.k.y, pp.r.z + s * pp.k.z};
            }
            // peeloffscattering (MonteCarloSimulation.cpp:319-363), unpolarized; replaced by the continuous
            // peel-off along the path when continuousScattering is on (:289-291)
            if (peel && !M.continuousScattering) {
                double wv[16];
                bool ok = true;
                if (Ncomp == 1) wv[0] = 1.0;
                else {
                    int m = M.grid.whichcell(pp.r.x, pp.r.y, pp.r.z);
                    if (m == -1) ok = false;
                    else {
                        double sum = 0;
                        for (int h = 0; h < Ncomp; h++) wv[h] = M.dust[h].mix.ksca[pp.ell] * M.rho[(size_t)m * Ncomp + h];
                        for (int h = 0; h < Ncomp; h++) sum += wv[h];
                        if (sum <= 0) ok = false;
                        else for (int h = 0; h < Ncomp; h++) wv[h] /= sum;
                    }
                }
                if (ok) {
                    for (size_t i = 0; i < M.instruments.size(); i++) {
                        const Instrument& ins = M.instruments[i];
                        double I = 0;
                        for (int h = 0; h < Ncomp; h++) {
                            double cosalpha = pp.k.x * ins.kobs[0] + pp.k.y * ins.kobs[1] + pp.k.z * ins.kobs[2];
                            double g = M.dust[h].mix.g[pp.ell];
                            double tt = 1.0 + g * g - 2 * g * cosalpha;
                            double w = wv[h] * ((1.0 - g) * (1.0 + g) / sqrt(tt * tt * tt));
                            I += w * 1.0;
                        }
                        Packet ppp = pp;
                        ppp.L = pp.L * I;
                        ppp.k = {ins.kobs[0], ins.kobs[1], ins.kobs[2]};
                        ppp.nscatt = pp.nscatt + 1;
                        detect(t, (int)i, ppp, tmp);
                    }
                }
            }
            // simulatescattering: DustSystem::randomMixForPosition + HG sampling (DustMix.cpp:609-613)
            int hmix = 0;
            if (Ncomp > 1) {
                int m = M.grid.whichcell(pp.r.x, pp.r.y, pp.r.z);
                if (m >= 0) {
                    std::vector<double> Xv(Ncomp + 1, 0.0);
                    for (int h = 0; h < Ncomp; h++) Xv[h + 1] = Xv[h] + M.dust[h].mix.ksca[pp.ell] * M.rho[(size_t)m * Ncomp + h];
                    double norm = Xv[Ncomp];
                    for (auto& v : Xv) v /= norm;
                    double X = rng.uniform();
                    int jl;
                    if (X < Xv[0]) jl = 0;
                    else { int lo = -1, hi = Ncomp; while (hi - lo > 1) { int jm = (hi + lo) >> 1; if (X < Xv[jm]) hi = jm; else lo = jm; } jl = lo; }
                    hmix = jl;
                }
            }
            double g = M.dust[hmix].mix.g[pp.ell];
            Vec3 knew;
            if (fabs(g) < 1e-6) knew = isotropic(rng);
            else {
                double f = ((1.0 - g) * (1.0 + g)) / (1.0 - g + 2.0 * g * rng.uniform());
                double costheta = (1.0 + g * g - f * f) / (2.0 * g);
                knew = rotated(rng, pp.k, costheta);
            }
            pp.nscatt++;
            pp.k = knew;
        }
    }

    // StellarSystem::launch + GeometricStellarComp::launch + PlummerGeometry/SpheGeometry sampling
    void launchStellar(Rng& rng, Packet& pp, int ell, double L) const {
        int N = (int)M.starL.size();
        int h = 0;
        double Lw = L;
        if (N > 1) {
            double X = rng.uniform();
            double xi = M.starEmissionBias;
            if (X < xi) h = std::max(0, std::min(N - 1, static_cast<int>(N * X / xi)));
            else {
                const std::vector<double>& Xv = M.starX[ell];
                double q = (X - xi) / (1.0 - xi);
                int n = (int)Xv.size();
                if (q < Xv[0]) h = 0;
                else { int lo = -1, hi = n - 1; while (hi - lo > 1) { int jm = (hi + lo) >> 1; if (q < Xv[jm]) hi = jm; else lo = jm; } h = lo; }
            }
            double Lh = M.starL[h][ell];
            if (Lh > 0) {
                double Lmean = M.starLtot[ell] / N;
                double weight = 1.0 / (1.0 - xi + xi * Lmean / Lh);
                Lw = L * weight;
            } else {
                pp = Packet{0., ell, {0, 0, 0}, {0, 0, 1}, 0, h};
                return;
            }
        }
        const Geometry& geo = M.starGeom[h];
        Vec3 pos;
        if (geo.kind == GeometryKind::Point) {
            pos = Vec3{0, 0, 0};  // PointGeometry::generatePosition: no draws
        } else if (geo.kind == GeometryKind::ExpDisk) {
            // ExpDiskGeometry::randomR / randomz, SepAxGeometry::generatePosition
            expDiskPosition(geo, rng, pos.x, pos.y, pos.z);
        } else if (geo.kind == GeometryKind::Sersic) {
            // SersicGeometry::randomradius, SpheGeometry::generatePosition
            sersicPosition(geo, rng, pos.x, pos.y, pos.z);
        } else {
            // PlummerGeometry::randomradius then SpheGeometry::generatePosition
            double t = pow(rng.uniform(), 1.0 / 3.0);
            double r = geo.c * t / sqrt((1.0 - t) * (1.0 + t));
            Vec3 d = isotropic(rng);
            pos = Vec3{r * d.x, r * d.y, r * d.z};
        }
        Vec3 k = isotropic(rng);
        pp = Packet{Lw, ell, pos, k, 0, h};
    }

    // the launch of dodustemissionchunk (biased cell choice, PanMonteCarloSimulation.cpp:296-325) and
    // of dodustselfabsorptionchunk (natural cell choice, :207-216): cell, random position in the cell
    // (Random::position(box), Random.cpp:226-234), isotropic direction; PhotonPackage::launch makes the
    // packet a dust packet (stellar = -1, PhotonPackage.cpp)
    void launchCell(Rng& rng, Packet& pp, int ell, const CellSources& src, double L, bool biased, double xi) const {
        int N = M.ncells();
        const double* Lv = &src.lv[(size_t)ell * N];
        const double* Xv = &src.cdf[(size_t)ell * (N + 1)];
        auto locateClip = [&](double x) {
            if (x < Xv[0]) return 0;
            int jl = -1, ju = N;
            while (ju - jl > 1) { int jm = (ju + jl) >> 1; if (x < Xv[jm]) ju = jm; else jl = jm; }
            return jl;
        };
        double X = rng.uniform();
        int m;
        double Lw = L;
        if (biased) {
            if (X < xi) m = std::max(0, std::min(N - 1, static_cast<int>(N * X / xi)));
            else m = locateClip((X - xi) / (1 - xi));
            double Lmean = src.ltot[ell] / N;
            double weight = 1.0 / (1 - xi + xi * Lmean / Lv[m]);
            Lw = L * weight;
        } else {
            m = locateClip(X);
        }
        Vec3 pos;
        if (M.grid.kind == GridKind::Voronoi) {
            // VoronoiMesh::randomPosition (VoronoiMesh.cpp:591-604)
            struct Src final : UniformSource {
                Rng& r;
                explicit Src(Rng& x) : r(x) {}
                double uniform() override { return r.uniform(); }
            } src(rng);
            voronoiRandomPosition(M.grid.vor, src, m, pos.x, pos.y, pos.z);
        } else {
            double b[6];
            M.grid.cellBox(m, b);
            double x = rng.uniform();
            double y = rng.uniform();
            double z = rng.uniform();
            pos = Vec3{b[0] + x * (b[3] - b[0]), b[1] + y * (b[4] - b[1]), b[2] + z * (b[5] - b[2])};
        }
        Vec3 k = isotropic(rng);
        pp = Packet{Lw, ell, pos, k, 0, -1};
    }
};

// one photon phase: which packets, where their absorption goes
struct PhaseSpec {
    int phase = ORACLE_PHASE_STELLAR;
    uint32_t tag = 0;                // Philox counter word 1: phase | cycle << 2 (the engine's convention)
    uint64_t Npp = 0;                // packets per wavelength (setChunkParams with one chunk)
    const CellSources* src = nullptr;
    std::vector<double>* labs = nullptr;
    bool store = false;
};

}  // namespace

struct OracleRun {
    std::unique_ptr<Model> model;
    Tallies tal;
    std::vector<double> labsDustTotals;  // Labsdusttot after every self-absorption cycle
    double seconds = 0;
    uint64_t packets = 0;
};

extern "C" {

const char* oracle_last_error(void) { return g_error.c_str(); }

void oracle_set_engine_attenuation(int mode) { g_engineAttenuation = (mode == 1 || mode == 2) ? mode : 0; }

void oracle_set_fill_hook(OracleFillHook hook, void* user) {
    g_fillUser = user;
    g_fillHook = hook;
}

void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) { philox(ctr, key, out); }

OracleRun* oracle_run(const char* ski, const char* datadir, int rngKind, int nthreads, double packages,
                      uint64_t seed, uint64_t packet_begin, uint64_t packet_end, int phases, const char* outprefix) {
    return oracle_run_shard(ski, datadir, rngKind, nthreads, packages, seed, packet_begin, packet_end, phases,
                            outprefix, 0, 1, nullptr, nullptr);
}

OracleRun* oracle_run_shard(const char* ski, const char* datadir, int rngKind, int nthreads, double packages,
                            uint64_t seed, uint64_t packet_begin, uint64_t packet_end, int phases,
                            const char* outprefix, int rank, int world, OracleReduceFn reduce, void* user) {
    try {
        if (world < 1 || rank < 0 || rank >= world) throw std::runtime_error("bad shard (rank, world)");
        if (world > 1 && (rngKind != ORACLE_RNG_PHILOX || packet_end))
            throw std::runtime_error("a shard needs Philox streams and no packet range");
        auto sum = [&](int tally, std::vector<double>& v) {
            if (world > 1 && reduce && !v.empty() && reduce(user, tally, v.data(), v.size()))
                throw std::runtime_error("the reduction failed");
        };
        auto run = std::make_unique<OracleRun>();
        // the MT stream must be seeded before setup, so the seed is read from the XML first
        unsigned long theSeed = seed ? (unsigned long)seed : readSkiSeed(ski);
        std::string dd = datadir && *datadir ? datadir : defaultDataDir();
        MTRandom mt(theSeed);
        run->model = std::make_unique<Model>(loadSki(ski, mt, dd));
        Model& M = *run->model;
        M.seed = theSeed;
        if (packages > 0) M.packages = packages;
        if (phases == 0) phases = ORACLE_PHASES_ALL;
        Sim sim(M);
        sim.initTallies(run->tal);
        const int Nl = M.wl.n();
        auto t0 = std::chrono::steady_clock::now();
        MTRng mtr(&mt);

        // shoots packet pk of a phase (global index: ell = pk / Npp, as in the engine)
        auto shoot = [&](const PhaseSpec& ph, Tallies& tl, Rng& rng, uint64_t pk, Path& p, Path& tmp,
                         uint64_t& count) {
            int ell = (int)(pk / ph.Npp);
            Sim::Packet pp;
            if (ph.phase == ORACLE_PHASE_STELLAR) {
                double L = M.starLtot[ell] / ph.Npp;
                if (!(L > 0)) return;  // dostellaremissionchunk skips the wavelength
                double Lthreshold = L / M.minWeightReduction;
                sim.launchStellar(rng, pp, ell, L);
                count++;
                if (pp.L > 0) {
                    if (M.hasDust) sim.lifeCycle(tl, rng, pp, Lthreshold, true, ph.store, ph.labs, p, tmp);
                    else
                        for (size_t q = 0; q < M.instruments.size(); q++) sim.detect(tl, (int)q, pp, tmp);
                }
            } else {
                double Ltot = ph.src->ltot[ell];
                if (!(Ltot > 0)) return;
                double L = Ltot / ph.Npp;  // Lem (dust emission) or L (self-absorption)
                double Lthreshold = L / M.minWeightReduction;
                bool emission = ph.phase == ORACLE_PHASE_DUST_EMISSION;
                sim.launchCell(rng, pp, ell, *ph.src, L, emission, M.dustEmissionBias);
                count++;
                sim.lifeCycle(tl, rng, pp, Lthreshold, emission, ph.store, ph.labs, p, tmp);
            }
        };
        // runs a phase over packets [pb, pe): MT mode in the reference's -t 1 order (chunk = wavelength,
        // packets in order), Philox mode over threads with one stream per packet
        // (pb, pe) index the phase's packets of this process: all of them, wavelength-slowest, or with a
        // shard (world > 1) the slice [lo, lo + cnt) of every wavelength (IdenticalAssigner.cpp:37-58)
        uint64_t sliceLo = 0, sliceCnt = 0;  // sliceCnt 0: no shard
        auto global = [&](const PhaseSpec& ph, uint64_t j) -> uint64_t {
            if (!sliceCnt) return j;
            const uint64_t ell = j / sliceCnt;
            return ell * ph.Npp + sliceLo + (j - ell * sliceCnt);
        };
        auto runPhase = [&](const PhaseSpec& ph, uint64_t pb, uint64_t pe) {
            Tallies& tl = run->tal;
            if (world > 1) {
                sliceLo = ph.Npp * (uint64_t)rank / (uint64_t)world;
                sliceCnt = ph.Npp * (uint64_t)(rank + 1) / (uint64_t)world - sliceLo;
                pb = 0;
                pe = sliceCnt * (uint64_t)Nl;
                if (!sliceCnt) return;
            }
            if (rngKind == ORACLE_RNG_MT) {
                Path p, tmp;
                p.v.reserve(1024);
                tmp.v.reserve(1024);
                Counts c;
                tCounts = &c;
                for (uint64_t pk = pb; pk < pe; pk++) shoot(ph, tl, mtr, pk, p, tmp, run->packets);
                tCounts = nullptr;
                c.mergeInto(tl);
                return;
            }
            int T = std::max(1, nthreads);
            tl.shared = true;
            std::vector<std::thread> th;
            std::atomic<uint64_t> next{pb};
            const uint64_t grain = 64;
            std::vector<std::string> errs(T);
            std::vector<uint64_t> cnt(T, 0);
            for (int w = 0; w < T; w++) {
                th.emplace_back([&, w] {
                    Counts c;
                    tCounts = &c;
                    struct Merge {  // on every exit of the worker
                        Counts& c;
                        Tallies& t;
                        ~Merge() { tCounts = nullptr; c.mergeInto(t); }
                    } merge{c, tl};
                    try {
                        PhiloxRng rng(theSeed, ph.tag);
                        Path p, tmp;
                        p.v.reserve(1024);
                        tmp.v.reserve(1024);
                        while (true) {
                            uint64_t b = next.fetch_add(grain);
                            if (b >= pe) break;
                            uint64_t e = std::min(pe, b + grain);
                            for (uint64_t j = b; j < e; j++) {
                                const uint64_t pk = global(ph, j);
                                rng.start(pk);
                                shoot(ph, tl, rng, pk, p, tmp, cnt[w]);
                            }
                        }
                    } catch (std::exception& ex) {
                        errs[w] = ex.what();
                    }
                });
            }
            for (auto& x : th) x.join();
            tl.shared = false;
            for (int w = 0; w < T; w++)
                if (!errs[w].empty()) throw std::runtime_error(errs[w]);
            for (int w = 0; w < T; w++) run->packets += cnt[w];
        };

        // ---- runstellaremission (MonteCarloSimulation.cpp:251-261)
        if (phases & ORACLE_PHASES_STELLAR) {
            PhaseSpec ph;
            ph.Npp = (uint64_t)std::ceil(M.packages);
            ph.store = M.hasDust && M.storeAbsorption;
            ph.labs = &run->tal.labs;
            uint64_t total = ph.Npp * (uint64_t)Nl;
            uint64_t pb = packet_begin, pe = packet_end ? std::min<uint64_t>(packet_end, total) : total;
            runPhase(ph, pb, pe);
            if (ph.store) sum(ORACLE_TALLY_LABS, run->tal.labs);  // PanDustSystem::sumResults(true)
        }
        // ---- rundustselfabsorption + rundustemission (PanMonteCarloSimulation::runSelf, .cpp:96-105)
        if ((phases & ORACLE_PHASES_DUST) && M.hasDust && M.dustEmission) {
            if (world > 1 && !reduce) throw std::runtime_error("sharded dust phases need a reducer");
            std::vector<PlanckTable> tables = planckTables(M);
            std::vector<double> lum;
            CellSources src;
            uint32_t cycleIndex = 0;
            if (M.selfAbsorption) {
                run->tal.labsDust.assign(run->tal.labs.size(), 0.0);
                SelfAbsorptionSchedule sched;
                sched.fixedCycles = M.cycles;
                while (sched.next()) {
                    // calculatedustemission, then Labsbolv = Labs(m), then rebootLabsdust
                    dustEmissionSpectra(M, tables, totalLabs(M, run->tal.labs, &run->tal.labsDust), lum);
                    cellSources(M, run->tal.labs, &run->tal.labsDust, lum, src);
                    std::fill(run->tal.labsDust.begin(), run->tal.labsDust.end(), 0.0);
                    PhaseSpec ph;
                    ph.phase = ORACLE_PHASE_DUST_SELFABS;
                    ph.tag = ORACLE_PHASE_DUST_SELFABS | (cycleIndex++ << 2);
                    ph.Npp = (uint64_t)std::ceil(M.packages * SelfAbsorptionSchedule::factor(sched.stage));
                    ph.src = &src;
                    ph.labs = &run->tal.labsDust;
                    ph.store = true;
                    runPhase(ph, 0, ph.Npp * (uint64_t)Nl);
                    sum(ORACLE_TALLY_DUST_LABS, run->tal.labsDust);  // Labsdusttot sums over processes
                    run->labsDustTotals.push_back(tableTotal(run->tal.labsDust));
                    sched.finishCycle(run->labsDustTotals.back());
                }
            }
            const std::vector<double>* dust = M.selfAbsorption ? &run->tal.labsDust : nullptr;
            dustEmissionSpectra(M, tables, totalLabs(M, run->tal.labs, dust), lum);
            cellSources(M, run->tal.labs, dust, lum, src);
            PhaseSpec ph;
            ph.phase = ORACLE_PHASE_DUST_EMISSION;
            ph.tag = ORACLE_PHASE_DUST_EMISSION;
            ph.Npp = (uint64_t)std::ceil(M.packages * M.emissionBoost);
            ph.src = &src;
            runPhase(ph, 0, ph.Npp * (uint64_t)Nl);
        }
        run->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (outprefix && *outprefix) {
            const std::vector<double>* dust = run->tal.labsDust.empty() ? nullptr : &run->tal.labsDust;
            writeOutputs(M, outprefix, run->tal.frames, run->tal.seds, totalLabs(M, run->tal.labs, dust));
            if (M.hasDust && M.writeCellsCrossed) writeCellsCrossed(M, outprefix, run->tal.crossed);
            if (M.hasDust && M.writeConvergence) {
                // DustSystem::writeconvergence (DustSystem.cpp:195-242): the paths from the origin along the
                // six half axes, DustGridPath::opticalDepth of DustSystem::density (DustSystem.cpp:925-931)
                const int Ncomp = (int)M.dust.size();
                auto density = [&](int m) {
                    double rho = 0;
                    if (m >= 0)
                        for (int h = 0; h < Ncomp; h++) rho += M.rho[(size_t)m * Ncomp + h];
                    return rho;
                };
                double sigma[3];
                Path p;
                for (int ax = 0; ax < 3; ax++) {
                    sigma[ax] = 0;
                    for (int sgn = 1; sgn >= -1; sgn -= 2) {
                        Vec3 k{0, 0, 0};
                        (ax == 0 ? k.x : ax == 1 ? k.y : k.z) = sgn;
                        sim.path(Vec3{0, 0, 0}, k, p);
                        double tau = 0;
                        for (auto& sg : p.v) tau += density(sg.m) * sg.ds;
                        sigma[ax] += tau;
                    }
                }
                writeConvergence(M, outprefix, sigma);
            }
        }
        return run.release();
    } catch (std::exception& ex) {
        g_error = ex.what();
        return nullptr;
    }
}

const double* oracle_labs(OracleRun* r, int* ncells, int* nlambda) {
    *ncells = r->model->ncells();
    *nlambda = r->model->wl.n();
    return r->tal.labs.empty() ? nullptr : r->tal.labs.data();
}

int oracle_num_instruments(OracleRun* r) { return (int)r->model->instruments.size(); }

int oracle_instrument(OracleRun* r, int i, const double** frames, const double** seds, int* nslots, int* nframe,
                      int* nlambda) {
    if (i < 0 || i >= (int)r->model->instruments.size()) return -1;
    const Instrument& ins = r->model->instruments[i];
    *frames = r->tal.frames[i].empty() ? nullptr : r->tal.frames[i].data();
    *seds = r->tal.seds[i].empty() ? nullptr : r->tal.seds[i].data();
    *nslots = ins.nslots();
    *nframe = ins.hasFrames() ? ins.nframe() : 0;
    *nlambda = r->model->wl.n();
    return 0;
}

const double* oracle_labs_dust(OracleRun* r) { return r->tal.labsDust.empty() ? nullptr : r->tal.labsDust.data(); }

int oracle_selfabs_cycles(OracleRun* r, const double** totals) {
    *totals = r->labsDustTotals.empty() ? nullptr : r->labsDustTotals.data();
    return (int)r->labsDustTotals.size();
}

int oracle_grid_paths(const char* ski, const char* datadir, int n, const double* rays, int maxseg, double* out,
                      int* nseg, int* ncells) {
    try {
        std::string dd = datadir && *datadir ? datadir : defaultDataDir();
        MTRandom mt(readSkiSeed(ski));
        Model M = loadSki(ski, mt, dd);
        if (!M.hasDust) throw std::runtime_error("the model has no dust grid");
        if (ncells) *ncells = M.ncells();
        Sim sim(M);
        Path p;
        for (int i = 0; i < n; i++) {
            const double* q = rays + 6 * (size_t)i;
            sim.path(Vec3{q[0], q[1], q[2]}, Vec3{q[3], q[4], q[5]}, p);
            const int ns = std::min<int>((int)p.v.size(), maxseg);
            nseg[i] = ns;
            for (int j = 0; j < ns; j++) {
                double* o = out + 7 * ((size_t)i * maxseg + j);
                if (p.v[j].m >= 0) M.grid.cellBox(p.v[j].m, o);
                else for (int k = 0; k < 6; k++) o[k] = NAN;
                o[6] = p.v[j].ds;
            }
        }
        return 0;
    } catch (const std::exception& e) {
        g_error = e.what();
        return -1;
    }
}

int oracle_dust_component(const char* ski, const char* datadir, int comp, double* nf, double* kext, double* lambda,
                          int* nlambda) {
    try {
        std::string dd = datadir && *datadir ? datadir : defaultDataDir();
        MTRandom mt(readSkiSeed(ski));
        Model M = loadSki(ski, mt, dd);
        if (comp < 0 || comp >= (int)M.dust.size()) throw std::runtime_error("no such dust component");
        const DustComp& d = M.dust[comp];
        *nf = d.nf;
        *nlambda = M.wl.n();
        for (int ell = 0; ell < M.wl.n(); ell++) {
            if (kext) kext[ell] = d.mix.kext[ell];
            if (lambda) lambda[ell] = M.wl.lambda[ell];
        }
        return 0;
    } catch (const std::exception& e) {
        g_error = e.what();
        return -1;
    }
}

int oracle_star_positions(const char* ski, const char* datadir, int comp, int n, uint64_t seed, double* out,
                          double* density) {
    try {
        std::string dd = datadir && *datadir ? datadir : defaultDataDir();
        MTRandom mt(readSkiSeed(ski));
        Model M = loadSki(ski, mt, dd);
        if (comp < 0 || comp >= (int)M.starGeom.size()) throw std::runtime_error("no such stellar component");
        const Geometry& geo = M.starGeom[comp];
        MTRandom mtr((unsigned long)seed);
        MTRng rng(&mtr);
        for (int i = 0; i < n; i++) {
            double* o = out + 3 * (size_t)i;
            if (geo.kind == GeometryKind::Point) {
                o[0] = o[1] = o[2] = 0.0;
            } else if (geo.kind == GeometryKind::ExpDisk) {
                expDiskPosition(geo, rng, o[0], o[1], o[2]);
            } else if (geo.kind == GeometryKind::Sersic) {
                sersicPosition(geo, rng, o[0], o[1], o[2]);
            } else {
                const double t = pow(rng.uniform(), 1.0 / 3.0);
                const double r = geo.c * t / sqrt((1.0 - t) * (1.0 + t));
                const Vec3 d = isotropic(rng);
                o[0] = r * d.x; o[1] = r * d.y; o[2] = r * d.z;
            }
            if (density) density[i] = geo.density(o[0], o[1], o[2]);
        }
        return 0;
    } catch (const std::exception& e) {
        g_error = e.what();
        return -1;
    }
}

double oracle_seconds(OracleRun* r) { return r->seconds; }
uint64_t oracle_packets(OracleRun* r) { return r->packets; }
uint64_t oracle_segments(OracleRun* r) { return r->tal.segments; }
void oracle_counts(OracleRun* r, uint64_t out[3]) {
    out[0] = r->tal.segFill;
    out[1] = r->tal.segPeel;
    out[2] = r->tal.absorbs;
}
int oracle_crossed(OracleRun* r, const uint64_t** hist) {
    int n = (int)r->tal.crossed.size();
    while (n > 0 && r->tal.crossed[n - 1] == 0) n--;
    *hist = r->tal.crossed.data();
    return n;
}
void oracle_free(OracleRun* r) { delete r; }

}  // extern "C"
