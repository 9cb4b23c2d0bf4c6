// pe_launch — MPI-free process launcher (the reference runs under mpirun /
// LSF, stage*/Этап*.pdf).  Spawns N ranks of a program on this node with
//   PE_RANK / PE_WORLD_SIZE / PE_LOCAL_RANK (and RANK / WORLD_SIZE / LOCAL_RANK)
//   PE_BOOTSTRAP_DIR  — a fresh directory for the RCCL unique-id handshake
// waits for all of them, and kills the whole job when one rank fails (the
// reference's checkCuda exit leaves MPI peers hanging — quirk A18).
// The launcher itself never touches the GPU; children exec immediately.
//   pe_launch -n 8 [--] prog args...
#include <signal.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

int main(int argc, char** argv) {
  int n = 1, i = 1;
  for (; i < argc; ++i) {
    if (!std::strcmp(argv[i], "-n") && i + 1 < argc) {
      n = std::atoi(argv[++i]);
    } else if (!std::strcmp(argv[i], "--")) {
      ++i;
      break;
    } else {
      break;
    }
  }
  if (i >= argc || n < 1) {
    std::fprintf(stderr, "usage: pe_launch -n N [--] prog args...\n");
    return 2;
  }
  char tmpl[] = "/tmp/pe_launch_XXXXXX";
  const char* dir = mkdtemp(tmpl);
  if (!dir) {
    std::perror("mkdtemp");
    return 2;
  }
  std::vector<pid_t> pids;
  for (int r = 0; r < n; ++r) {
    pid_t pid = fork();
    if (pid < 0) {
      std::perror("fork");
      return 2;
    }
    if (pid == 0) {
      setpgid(0, 0);
      const std::string rs = std::to_string(r), ns = std::to_string(n);
      setenv("PE_RANK", rs.c_str(), 1);
      setenv("PE_WORLD_SIZE", ns.c_str(), 1);
      setenv("PE_LOCAL_RANK", rs.c_str(), 1);
      setenv("RANK", rs.c_str(), 1);
      setenv("WORLD_SIZE", ns.c_str(), 1);
      setenv("LOCAL_RANK", rs.c_str(), 1);
      setenv("PE_BOOTSTRAP_DIR", dir, 1);
      execvp(argv[i], argv + i);
      std::perror("execvp");
      _exit(127);
    }
    pids.push_back(pid);
  }
  int rc = 0, alive = n;
  while (alive > 0) {
    int status = 0;
    const pid_t p = wait(&status);
    if (p < 0) break;
    --alive;
    const int code = WIFEXITED(status) ? WEXITSTATUS(status) : 128 + WTERMSIG(status);
    if (code != 0 && rc == 0) {
      rc = code;
      std::fprintf(stderr, "[pe_launch] rank pid %d failed (code %d); terminating the job\n", int(p), code);
      for (pid_t q : pids)
        if (q != p) kill(-q, SIGTERM);
    }
  }
  std::string cleanup = std::string(dir) + "/rccl_uid";
  unlink(cleanup.c_str());
  rmdir(dir);
  return rc;
}
