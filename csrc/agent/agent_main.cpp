// agent_main.cpp — `dpu-cp-agent`: the node control agent as a standalone native daemon.
//
// Reference: octep_cp_agent main.c (SURVEY NAT1): `octep_cp_agent <file.cfg> -- [opts]`, parse the
// config, init, announce fw-ready, loop until SIGINT/SIGTERM, uninit.  Options here:
//   dpu-cp-agent <file.cfg> [--mbox PATH] [--size BYTES] [--max-msgs N] [--plugin-port P]
// Defaults: mailbox /var/run/dpu-daemon/ctrl-mbox (32 KiB), 6 messages per PF per iteration,
// plugin relay on 49500 (-1 disables).
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <thread>

#include "agent.h"
#include "plugin_server.h"
#include "soc.h"

static volatile std::sig_atomic_t g_stop = 0;
static void on_signal(int) { g_stop = 1; }

int main(int argc, char** argv) {
  if (argc < 2 || !std::strcmp(argv[1], "-h") || !std::strcmp(argv[1], "--help")) {
    std::fprintf(stderr, "usage: %s <file.cfg> [--mbox PATH] [--size BYTES] [--max-msgs N] [--plugin-port P]\n"
                         "       %s --list-gpus [SYS_ROOT]\n", argv[0], argv[0]);
    return 2;
  }
  if (!std::strcmp(argv[1], "--list-gpus")) {  // soc detection (the reference's soc.c role)
    const char* root = argc > 2 ? argv[2] : "/";
    for (const agent::GpuInfo& g : agent::detect_gpus(root))
      std::printf("{\"node\": %d, \"model\": \"%s\", \"gfx\": \"%s\", \"cus\": %u, \"xcc\": %u, \"vram_gib\": %.0f, "
                  "\"numa\": %d, \"pci\": \"%s\"}\n", g.node, g.model_name.c_str(), g.gfx_arch.c_str(), g.cu_count,
                  g.num_xcc, g.vram_bytes / 1073741824.0, g.numa_node, g.pci.c_str());
    return 0;
  }
  std::string cfg_path = argv[1], mbox = "/var/run/dpu-daemon/ctrl-mbox";
  uint32_t size = 32768;
  int max_msgs = 6, plugin_port = agent::PluginServer::kDefaultPort;
  for (int i = 2; i < argc; ++i) {
    const std::string a = argv[i];
    auto next = [&](const char* what) -> const char* {
      if (i + 1 >= argc) { std::fprintf(stderr, "missing value for %s\n", what); std::exit(2); }
      return argv[++i];
    };
    if (a == "--") continue;
    if (a == "--mbox") mbox = next("--mbox");
    else if (a == "--size") size = (uint32_t)std::strtoul(next("--size"), nullptr, 0);
    else if (a == "--max-msgs") max_msgs = std::atoi(next("--max-msgs"));
    else if (a == "--plugin-port") plugin_port = std::atoi(next("--plugin-port"));
    else { std::fprintf(stderr, "unknown option %s\n", a.c_str()); return 2; }
  }
  std::ifstream f(cfg_path);
  if (!f) { std::fprintf(stderr, "cannot read %s\n", cfg_path.c_str()); return 1; }
  std::stringstream ss;
  ss << f.rdbuf();
  try {
    agent::Agent ag(mbox, agent::build_agent_config(agent::parse_config(ss.str())), size, max_msgs);
    std::signal(SIGINT, on_signal);
    std::signal(SIGTERM, on_signal);
    ag.start(plugin_port);
    std::printf("dpu-cp-agent: ready (mbox %s, %zu functions, plugin port %d)\n", mbox.c_str(), ag.functions().size(),
                ag.plugin_port());
    std::fflush(stdout);
    while (!g_stop) std::this_thread::sleep_for(std::chrono::milliseconds(50));
    ag.stop();
  } catch (const std::exception& e) {
    std::fprintf(stderr, "dpu-cp-agent: %s\n", e.what());
    return 1;
  }
  std::printf("dpu-cp-agent: stopped\n");
  return 0;
}
