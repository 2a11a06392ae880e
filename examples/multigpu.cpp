// examples/multigpu.cpp — SURVEY §8(e) from a C++ host, no Python: pixel-row tiles on
// every GPU and one RCCL gather, through the C ABI (include/rtmi.h).
//
//   ./multigpu [width=512] [height=512] [spp=32] [gpus=1] [row_block=2]
//
// 1. One process per GPU (the scaling shape): the parent forks `gpus` children BEFORE
//    anything touches the GPU. Child k opens device k, renders its tiles with
//    rt_render_device and joins rt_gather_rows (one ncclGather + the device
//    de-interleave on rank 0); rank 0 publishes the unique id through a file and
//    writes the assembled frame back for the parent.
// 2. One process driving every GPU: rt_render_multi over contexts on devices 0..gpus-1.
// Both frames must equal a single-device rt_render bit for bit (the RNG is keyed by
// the global pixel, and every rank folds samples with the frame's sub-stream count).
#include <hip/hip_runtime_api.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rtmi.h"

namespace {

const char* kScene = RTMI_ASSETS "/scenes/cornellbox1.yaml";
const char* kModels = RTMI_ASSETS "/models";

bool ok(rt_status s, rt_ctx* c, const char* what) {
    if (s == RT_OK) return true;
    std::fprintf(stderr, "%s failed: %d (%s)\n", what, s, c ? rt_last_error(c) : "");
    return false;
}

rt_ctx* open_scene(int device, int w, int h) {
    rt_ctx* c = nullptr;
    if (rt_create(device, &c) != RT_OK) return nullptr;
    if (!ok(rt_load_yaml_scene(c, kScene, kModels, w, h), c, "rt_load_yaml_scene") ||
        !ok(rt_commit(c), c, "rt_commit")) {
        rt_destroy(c);
        return nullptr;
    }
    return c;
}

rt_render_params frame_params(int w, int h, int spp, int row_block, int rank, int world) {
    rt_render_params p{};
    p.width = w;
    p.height = h;
    p.spp = spp;
    p.max_depth = 8;
    p.seed = 1984;
    p.row_block = row_block;
    p.row_rank = rank;
    p.row_world = world;
    p.lanes_per_pixel = 0;
    p.integrator = RT_INTEGRATOR_RAYCOLOR;
    return p;
}

// Child process of rank `rank`: render this rank's tiles, gather to rank 0.
int rank_main(int rank, int world, int w, int h, int spp, int rb, const std::string& dir) {
    rt_ctx* c = open_scene(rank, w, h);
    if (!c) return 10;
    const std::string id_file = dir + "/nccl.id", frame_file = dir + "/frame.f32";
    uint8_t id[128];
    if (rank == 0) {
        if (!ok(rt_comm_unique_id(id), c, "rt_comm_unique_id")) return 11;
        const std::string tmp = id_file + ".tmp";
        FILE* f = std::fopen(tmp.c_str(), "wb");
        if (!f || std::fwrite(id, 1, 128, f) != 128 || std::fclose(f) != 0) return 12;
        std::rename(tmp.c_str(), id_file.c_str());
    } else {
        for (int t = 0;; ++t) {  // rank 0 publishes the id (bounded wait)
            FILE* f = std::fopen(id_file.c_str(), "rb");
            if (f) {
                const size_t n = std::fread(id, 1, 128, f);
                std::fclose(f);
                if (n == 128) break;
            }
            if (t > 6000) return 13;
            usleep(10000);
        }
    }
    void* comm = nullptr;
    if (!ok(rt_comm_init(c, id, world, rank, &comm), c, "rt_comm_init")) return 14;
    const rt_render_params p = frame_params(w, h, spp, rb, rank, world);
    const size_t tile_floats = (size_t)rt_max_tile_rows(h, rb, world) * w * 3;
    const size_t frame_floats = (size_t)w * h * 3;
    float *tile = nullptr, *frame = nullptr;
    if (hipMalloc((void**)&tile, tile_floats * sizeof(float)) != hipSuccess) return 15;
    if (rank == 0 && hipMalloc((void**)&frame, frame_floats * sizeof(float)) != hipSuccess) return 15;
    if (!ok(rt_render_device(c, &p, tile, nullptr), c, "rt_render_device") ||
        !ok(rt_gather_rows(c, comm, &p, rank, world, tile, frame, nullptr), c, "rt_gather_rows"))
        return 16;
    if (hipDeviceSynchronize() != hipSuccess) return 17;
    if (rank == 0) {
        std::vector<float> host(frame_floats);
        if (hipMemcpy(host.data(), frame, frame_floats * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
            return 18;
        FILE* f = std::fopen(frame_file.c_str(), "wb");
        if (!f || std::fwrite(host.data(), sizeof(float), frame_floats, f) != frame_floats || std::fclose(f) != 0)
            return 19;
    }
    rt_sync_stats(c, nullptr);
    (void)hipFree(tile);
    (void)hipFree(frame);
    rt_comm_destroy(comm);
    rt_destroy(c);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    const int w = argc > 1 ? atoi(argv[1]) : 512, h = argc > 2 ? atoi(argv[2]) : 512;
    const int spp = argc > 3 ? atoi(argv[3]) : 32, gpus = argc > 4 ? atoi(argv[4]) : 1;
    const int rb = argc > 5 ? atoi(argv[5]) : 2;
    if (w < 2 || h < 2 || spp < 1 || gpus < 1 || gpus > 8 || rb < 1) {
        std::fprintf(stderr, "usage: multigpu [width] [height] [spp] [gpus 1-8] [row_block]\n");
        return 2;
    }
    char tmpl[] = "/tmp/rtmi_multigpu_XXXXXX";
    if (!mkdtemp(tmpl)) return 3;
    const std::string dir = tmpl;

    // 1. one process per GPU: fork first, before this process touches the GPU
    std::vector<pid_t> kids;
    for (int k = 0; k < gpus; ++k) {
        const pid_t pid = fork();
        if (pid < 0) return 4;
        if (pid == 0) _exit(rank_main(k, gpus, w, h, spp, rb, dir));
        kids.push_back(pid);
    }
    bool kids_ok = true;
    for (pid_t pid : kids) {
        int status = 0;
        waitpid(pid, &status, 0);
        if (!WIFEXITED(status) || WEXITSTATUS(status) != 0) {
            std::fprintf(stderr, "rank process %d failed (status %d)\n", (int)pid, status);
            kids_ok = false;
        }
    }
    const size_t frame_floats = (size_t)w * h * 3;
    std::vector<float> gathered(frame_floats);
    if (kids_ok) {
        FILE* f = std::fopen((dir + "/frame.f32").c_str(), "rb");
        kids_ok = f && std::fread(gathered.data(), sizeof(float), frame_floats, f) == frame_floats;
        if (f) std::fclose(f);
    }
    std::remove((dir + "/frame.f32").c_str());
    std::remove((dir + "/nccl.id").c_str());
    rmdir(dir.c_str());

    // 2. one process, every GPU: rt_render_multi, and the single-device reference
    std::vector<rt_ctx*> ctxs;
    for (int k = 0; k < gpus; ++k) {
        rt_ctx* c = open_scene(k, w, h);
        if (!c) return 5;
        ctxs.push_back(c);
    }
    std::vector<float> single(frame_floats), multi(frame_floats);
    rt_render_params p = frame_params(w, h, spp, rb, 0, 1);
    if (!ok(rt_render(ctxs[0], &p, single.data()), ctxs[0], "rt_render")) return 6;
    if (!ok(rt_render_multi(ctxs.data(), gpus, &p, multi.data()), ctxs[0], "rt_render_multi")) return 7;
    rt_render_stats st{};
    rt_sync_stats(ctxs[0], &st);
    const bool multi_ok = std::memcmp(single.data(), multi.data(), frame_floats * sizeof(float)) == 0;
    const bool gather_ok = kids_ok && std::memcmp(single.data(), gathered.data(), frame_floats * sizeof(float)) == 0;
    std::printf("render_multi %s (%d GPU%s, exchange %s)\n", multi_ok ? "ok" : "MISMATCH", gpus,
                gpus > 1 ? "s" : "", st.gather == RT_GATHER_RCCL ? "ncclGather" : "device copies");
    std::printf("gather_rows %s (%d process%s, one ncclGather)\n", gather_ok ? "ok" : "FAILED", gpus,
                gpus > 1 ? "es" : "");
    for (rt_ctx* c : ctxs) rt_destroy(c);
    return multi_ok && gather_ok ? 0 : 1;
}
